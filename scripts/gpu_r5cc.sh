# Round 5: the co-residency change (r5bb: accumulation prefetch 1 group + Adam folding replicas one at a time,
# +1.8 % in 3 of 3 pairs) re-measured with more pairs, and the march at 5 waves per SIMD (launch bound 96 VGPRs,
# 6 VGPRs spilled) alone and with it.
# usage: gpurun -- bash scripts/gpu_r5cc.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5cc}
bash scripts/ab_env.sh $T 5 "||--steps 600" "lib_co1||--steps 600" "lib_m5||--steps 600" "lib_co1m5||--steps 600"
