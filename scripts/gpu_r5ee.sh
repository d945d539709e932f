# Round 5: r5dd's two +0.8-0.9 % candidates combined (accumulation without the Adam-state prefetch, coarse grid
# capped at 512 blocks), 6 alternating pairs against the default.
# usage: gpurun -- bash scripts/gpu_r5ee.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5ee}
bash scripts/ab_env.sh $T 6 "||--steps 600" "lib_pc||--steps 600"
