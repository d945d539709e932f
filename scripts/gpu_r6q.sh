# Round 6: quality at the reference schedule, 3 seeds per mode: product defaults vs exact mode.
# usage: gpurun --timeout 1200 -- bash scripts/gpu_r6q.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r6q}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 1100 python -u scripts/quality_30k.py --seeds 4,5,6 > $OUT/quality_3seeds.json 2> $OUT/quality_3seeds.err || { tail -30 $OUT/quality_3seeds.err; exit 1; }
cat $OUT/quality_3seeds.json
