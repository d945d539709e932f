# Round 5: r5gg (coarse grid 256 / 512 / 1024) then the per-wave timeline of the final tree (r5tl).
# usage: gpurun -- bash scripts/gpu_r5hh.sh
set -e
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r5tl.sh r5tl
bash scripts/gpu_r5gg.sh r5gg
