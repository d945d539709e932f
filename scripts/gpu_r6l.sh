# Round 6: capture order of the step's forks, single bits (NGP_MAIN_FIRST 2 / 4 / 6 vs the default), 4 reps.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/ab_env.sh r6l 4 "||" "|NGP_MAIN_FIRST=2|" "|NGP_MAIN_FIRST=4|" "|NGP_MAIN_FIRST=6|"
