# Round 5: the accumulation without the Adam-state prefetch (93 VGPRs: two Adam waves per SIMD fit beside it, the
# fused buckets' p / m / v then read at the flush) against the adopted one-group prefetch (105 VGPRs); and, now that
# the coarse levels' Adam no longer waits for the accumulation (the coarse kernel has ~40 us of slack), the coarse
# kernel's grid capped at 512 / 1024 blocks, so the record write beside it is slowed less by its atomics.
# usage: gpurun -- bash scripts/gpu_r5dd.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5dd}
bash scripts/ab_env.sh $T 5 "||--steps 600" "lib_pf0||--steps 600" "lib_cc512||--steps 600" "lib_cc1024||--steps 600"
