set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dense
timeout -k 10 400 python -u -m pytest tests/test_field_gpu.py tests/test_trainer_gpu.py tests/test_ddp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dense/pytest.log 2>&1
bash scripts/gpu_ab.sh ab_dense "NGP_DENSE_IN_ACCUM=0" "NGP_DENSE_IN_ACCUM=1" 3
