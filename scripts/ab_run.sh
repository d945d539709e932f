set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/acc2
timeout -k 10 400 python -u -m pytest tests/test_trainer_gpu.py tests/test_field_gpu.py -x -v --timeout 120 --timeout-method thread -k "fused_adam or binned or replicated" > gpurun_out/acc2/pytest.log 2>&1
bash scripts/gpu_abn.sh ab_acc2 3 "NGP_AMD_LIB=build_ab/base.so" "NGP_X=1"
