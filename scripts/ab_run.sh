set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/b12
NGP_AMD_LIB=build_ab/b12.so timeout -k 10 400 python -u -m pytest tests/test_trainer_gpu.py tests/test_field_gpu.py -x -v --timeout 120 --timeout-method thread -k "fused_adam or binned" > gpurun_out/b12/pytest.log 2>&1
bash scripts/gpu_abn.sh ab_b12 3 "NGP_X=0" "NGP_AMD_LIB=build_ab/b12.so"
