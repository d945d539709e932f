set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/rt
timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py tests/test_trainer_gpu.py tests/test_golden_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rt/pytest.log 2>&1
bash scripts/gpu_abn.sh ab_rt 3 "NGP_AMD_LIB=build_ab/base.so" "NGP_X=1"
