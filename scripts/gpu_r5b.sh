# Round 5, second box: the GPU suite (LDS-merged coarse scatter, probes, pre-encoded round 1, captured
# data-parallel step, drop-in FusedAdam / loop, world-1 RCCL), then alternating A/Bs:
#   coarse modes (0 = per-wave merge, 1 = LDS 64-sample tiles, 2 = LDS 128-sample tiles) x pre-encode
#   the emulated world-8 step, K = 2 / 4 fine buckets, captured vs segmented, against single-process
# usage: gpurun -- bash scripts/gpu_r5b.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5b}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash scripts/ab_env.sh $T/ab 2 "|NGP_COARSE_LDS=0 NGP_PRE_COARSE=0|--steps 400" "|NGP_COARSE_LDS=1 NGP_PRE_COARSE=0|--steps 400" \
    "|NGP_COARSE_LDS=2 NGP_PRE_COARSE=0|--steps 400" "|NGP_COARSE_LDS=1 NGP_PRE_COARSE=1|--steps 400"
bash scripts/ab_env.sh $T/dp 1 "||--steps 300" "||--steps 300 --emulate-dp 8 --dp-fine-buckets 2" \
    "||--steps 300 --emulate-dp 8 --dp-fine-buckets 4" "|NGP_DP_CAPTURE=0|--steps 300 --emulate-dp 8 --dp-fine-buckets 2"
