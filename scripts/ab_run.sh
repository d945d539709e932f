set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/wf
NGP_WRITE_FIRST=1 timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -x -v --timeout 120 --timeout-method thread -k "fused_adam or step" > gpurun_out/wf/pytest.log 2>&1
bash scripts/gpu_abn.sh ab_wf 3 "NGP_WRITE_FIRST=0" "NGP_WRITE_FIRST=1"
