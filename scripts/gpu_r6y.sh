# Round 6: the HIP runtime's graph-queue count (DEBUG_HIP_FORCE_GRAPH_QUEUES) for the step graph; alternating
# 1000-step windows (the default = unset)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/ab_env.sh r6y 2 "||" "|DEBUG_HIP_FORCE_GRAPH_QUEUES=1|" "|DEBUG_HIP_FORCE_GRAPH_QUEUES=2|" "|DEBUG_HIP_FORCE_GRAPH_QUEUES=4|"
