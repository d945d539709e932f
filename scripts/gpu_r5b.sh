# Round 5, second box: the GPU suite on the LDS-merged coarse scatter + probes + drop-in tests, then
# an alternating A/B of the coarse modes (0 = per-wave merge, 1 = LDS 64-sample tiles, 2 = LDS
# 128-sample tiles).  usage: gpurun -- bash scripts/gpu_r5b.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5b}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash scripts/ab_env.sh $T/ab 2 "|NGP_COARSE_LDS=0|--steps 400" "|NGP_COARSE_LDS=1|--steps 400" "|NGP_COARSE_LDS=2|--steps 400"
