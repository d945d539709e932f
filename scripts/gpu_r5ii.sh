# Round 5: the pre-encode's start after the MLP + coarse Adam.  r5tl: it started ~12 us after the Adam's last wave
# (its graph node also waited on the march queue).  NGP_PRE_WAIT=pre: that wait on the pre-encode (as before);
# default: on the coarse kernel, which waits on the main stream anyway.  lib_ab512: + the replica-folding Adam as
# a 512-block grid-stride launch (2 waves per SIMD, the room beside the accumulation) instead of 2995 blocks.
# Then the per-wave timeline of the default.
# usage: gpurun -- bash scripts/gpu_r5ii.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5ii}
bash scripts/ab_env.sh $T 5 "|NGP_PRE_WAIT=pre|--steps 600" "||--steps 600" "lib_ab512||--steps 600"
bash scripts/gpu_r5tl.sh ${T}_tl
