# Round 6: the coarse hash kernel's grid (512 blocks since r5ff) now that the side chain (coarse -> Adam ->
# pre-encode) ends after the accumulation (r6final wave timeline); alternating 1000-step windows.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/ab_env.sh r6n 3 "||" "lib_cb1024||" "lib_cb2048||" "lib_cb256||"
