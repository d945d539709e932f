# Round 4: kernel statistics + one-step timelines of the default step (rocprofv3 kernel trace of a short bench).
# usage: gpurun -- bash scripts/gpu_r4k.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4s}; mkdir -p $OUT
Q="--psnr-views 0 --no-cpu-baseline --quality-steps 0 --no-oracle-quality --infer-frames 0 --breakdown-steps 1"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr" -o run -f csv -- python3 bench.py --steps 200 --warmup 5 $Q \
    > "$OUT/b.json" 2> "$OUT/b.err"
python3 scripts/kstats.py "$OUT/tr/run_kernel_trace.csv" 200 > $OUT/kstats.txt 2>&1 || true
for b in 10 11 12; do python3 scripts/timeline.py "$OUT/tr/run_kernel_trace.csv" 20 $b; done > "$OUT/timeline.txt"
rm -rf "$OUT/tr"
head -22 $OUT/kstats.txt; head -34 $OUT/timeline.txt
