# Round 5: the replica-folding MLP + coarse Adam as a grid-stride launch of 512 / 1024 blocks (the room beside the
# accumulation holds ~2 of its waves per SIMD) vs one float4 group per lane (2995 blocks), 6 pairs on the final tree.
# usage: gpurun -- bash scripts/gpu_r5nn.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5nn}
bash scripts/ab_env.sh $T 6 "||--steps 600" "lib_ab512||--steps 600" "lib_ab1024||--steps 600"
