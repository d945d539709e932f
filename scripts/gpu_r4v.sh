# Round 4: two steps per graph replay (the bench default) vs one, on the final schedule (A/B).  usage: gpurun -- bash scripts/gpu_r4v.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/ab_env.sh ${1:-r4pair}/ab 3 "||" "|| --no-pair-steps"
