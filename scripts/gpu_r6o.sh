# Round 6: where the next batch's march forks off the step, re-measured with the one-round march (r4's
# verdict "r1" was measured with the two-round march); alternating 1000-step windows.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/ab_env.sh r6o 3 "||" "|NGP_MARCH_AT_AB=start|" "|NGP_MARCH_AT_AB=fwd|" "|NGP_MARCH_AT_AB=mlp|"
