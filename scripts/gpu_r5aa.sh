# Round 5: where the atomic / binned split of the hash backward sits now (bin_level_lo 8 / 7 / 6): fewer coarse
# atomic levels shorten the coarse kernel and its Adam (which waits for the accumulation's blocks), at the cost of
# more buckets in the accumulation.
# usage: gpurun -- bash scripts/gpu_r5aa.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5aa}
bash scripts/ab_env.sh $T 2 "||--steps 600" "||--steps 600 --bin-level-lo 7" "||--steps 600 --bin-level-lo 6"
