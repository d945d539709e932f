# Round 4: the one-launch row forward (NGP_ROW_FWD=1): its tests, an alternating A/B against the
# two-round default, and a kernel trace + timeline of the row variant.  usage: gpurun -- bash scripts/gpu_r4g.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4g}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 3 $OUT/pytest.log
grep -E "evaluated samples|passed|failed" $OUT/pytest.log | tail -6 || true
bash scripts/ab_env.sh ${1:-r4g}/ab 3 "|NGP_ROW_FWD=0|" "||" "|NGP_ROW_FWD=2|" "|NGP_STEP_TICKET=1|"
Q="--psnr-views 0 --no-cpu-baseline --quality-steps 0 --no-oracle-quality --infer-frames 0 --breakdown-steps 1"
NGP_ROW_FWD=${ROWMODE:-2} timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr" -o run -f csv -- python3 bench.py --steps 200 --warmup 5 $Q \
    > "$OUT/b.json" 2> "$OUT/b.err"
python3 scripts/kstats.py "$OUT/tr/run_kernel_trace.csv" 200 > $OUT/kstats_rows.txt 2>&1 || true
for b in 10 11 12; do python3 scripts/timeline.py "$OUT/tr/run_kernel_trace.csv" 20 $b; done > "$OUT/timeline_rows.txt"
rm -rf "$OUT/tr"
head -16 $OUT/kstats_rows.txt; head -32 $OUT/timeline_rows.txt
