set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp


bash scripts/ab_garden.sh garden3 2 "" "--bin-merge-hi 8" "--bin-merge-hi 12" "--bin-level-lo 4"
