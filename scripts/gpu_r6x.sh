# Round 6 vs round 5, whole trees alternated on one box (abtree_r5 = the round-5 final commit, built in place):
# 600-step windows, the bench's defaults otherwise.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/ab_trees.sh r6x 5 ".||" "abtree_r5||"
