# Round 5: the fork-point A/B (r5kk), then the final check of the tree (gpu_r5_final.sh).
# usage: gpurun -- bash scripts/gpu_r5ll.sh
set -e
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r5kk.sh r5kk
bash scripts/gpu_r5_final.sh r5k
