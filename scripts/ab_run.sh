set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_abn.sh ab_rep3 2 "NGP_COARSE_REP=8" "NGP_COARSE_REP_LEVELS=5" "NGP_COARSE_REP_LEVELS=6" "NGP_COARSE_REP=16"
