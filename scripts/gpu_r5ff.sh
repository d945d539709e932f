# Round 5: the pre-encoded round 1 revived (r5f: round 1 61 -> 47 us, but the pre-encode waited behind the
# accumulation's register-full blocks) now that the accumulation leaves room beside it: the next batch's first
# chunks' levels 0-7 encoded after the MLP + coarse Adam, beside the accumulation.  lib_pcp = the accumulation
# without the Adam-state prefetch (93 VGPRs: the pre-encode's 67 + the Adam's 55 fit beside its 4 waves per SIMD)
# + the coarse grid capped at 512 blocks (r5ee: that pair +1.2 %, 5 of 6).  NGP_PRE_COARSE=0: round 1 gathers all.
# usage: gpurun -- bash scripts/gpu_r5ff.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5ff}
bash scripts/ab_env.sh $T 5 "|NGP_PRE_COARSE=0|--steps 600" "||--steps 600" "lib_pcp|NGP_PRE_COARSE=0|--steps 600" "lib_pcp||--steps 600"
