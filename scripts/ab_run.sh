set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dense2
timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -x -v --timeout 120 --timeout-method thread -k "dense or fused_adam" > gpurun_out/dense2/pytest.log 2>&1
