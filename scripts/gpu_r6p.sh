# Round 6: the march's blocks per CU capped by LDS padding (8 = the default, 64 VGPRs; 7 / 6 / 5 leave register
# file room for round 2's and the composite's waves beside it); alternating 1000-step windows.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/ab_env.sh r6p 3 "||" "lib_mlds7||" "lib_mlds6||" "lib_mlds5||"
