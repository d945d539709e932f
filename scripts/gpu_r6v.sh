# Round 6: the accumulation's blocks waiting for the coarse kernel's waves to leave (93 VGPRs x 4 waves per SIMD
# + the coarse waves' 64 exceed the register file where 3+ coarse waves share a SIMD): the accumulation capped
# at 80 VGPRs (6 waves/EU bound, 12 spilled), alternating 1000-step windows
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/ab_env.sh r6v 3 "||" "lib_acc6||"
