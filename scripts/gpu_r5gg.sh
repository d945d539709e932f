# Round 5: the training step's coarse-kernel grid (COARSE_BLOCKS 512, adopted in r5ff) against 256 and 1024 blocks
# on the final tree (pre-encoded round 1, prefetch-free accumulation).
# usage: gpurun -- bash scripts/gpu_r5gg.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5gg}
bash scripts/ab_env.sh $T 5 "||--steps 600" "lib_cb256||--steps 600" "lib_cb1024||--steps 600"
