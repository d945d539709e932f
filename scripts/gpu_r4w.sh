# Round 4: march fork point x march grid cap (A/B).  usage: gpurun -- bash scripts/gpu_r4w.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/ab_env.sh ${1:-r4mx}/ab ${REPS:-3} "||" "|NGP_MARCH_BLOCKS=1024|"
