# Round 6: gpu_r6f.sh (slot-layout march: suite, smoke, skip_cost, A/B vs dense) then gpu_r6e.sh (drop-in, driver cmd).
set -e
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r6f.sh ${1:-r6g}
bash scripts/gpu_r6e.sh ${1:-r6g}e
