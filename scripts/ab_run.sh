set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/cf0
NGP_CHUNK_FIRST=0 timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -x -v --timeout 120 --timeout-method thread -k "chunked or step or exact" > gpurun_out/cf0/pytest.log 2>&1
bash scripts/gpu_abn.sh ab_cf 2 "NGP_CHUNK_FIRST=64" "NGP_CHUNK_FIRST=0" "NGP_CHUNK_FIRST=96" "NGP_CHUNK_FIRST=48"
