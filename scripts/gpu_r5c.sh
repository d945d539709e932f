# Round 5: coarse scatter modes after batching the LDS table probes, pre-encoded round 1 on the
# default coarse path.  usage: gpurun -- bash scripts/gpu_r5c.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5c}
bash scripts/ab_env.sh $T/ab 2 "|NGP_COARSE_LDS=0 NGP_PRE_COARSE=0|--steps 400" "|NGP_COARSE_LDS=0 NGP_PRE_COARSE=1|--steps 400" \
    "|NGP_COARSE_LDS=1 NGP_PRE_COARSE=1|--steps 400"
