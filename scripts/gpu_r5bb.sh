# Round 5: the MLP + coarse Adam beside the accumulation -- its waves wait ~60 us for the accumulation's whole-CU
# blocks (16 waves x 128 VGPRs).  lib_co1: accumulation prefetch 1 group (105 VGPRs) + Adam folding replicas one at
# a time (60 VGPRs): one Adam wave per SIMD fits beside the accumulation; lib_pf1: the prefetch change alone.
# usage: gpurun -- bash scripts/gpu_r5bb.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5bb}
bash scripts/ab_env.sh $T 3 "||--steps 600" "lib_co1||--steps 600" "lib_pf1||--steps 600"
