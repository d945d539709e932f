# Round 6: fewer hardware queues per process than HIP's default 4 (8 and 16 measured 36-49 % slower, r6j).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6k; mkdir -p $OUT
bash scripts/ab_env.sh r6k 3 "||" "|GPU_MAX_HW_QUEUES=2|" "|GPU_MAX_HW_QUEUES=3|" "|GPU_MAX_HW_QUEUES=2 NGP_MAIN_FIRST=6|" "|GPU_MAX_HW_QUEUES=1|"
