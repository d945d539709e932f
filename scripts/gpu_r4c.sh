# Round 4: one-step timelines of the product step and of the emulated world-8 data-parallel step
# (rocprofv3 kernel traces of the bench).  usage: gpurun -- bash scripts/gpu_r4c.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4c}; mkdir -p $OUT
Q="--psnr-views 0 --no-cpu-baseline --quality-steps 0 --no-oracle-quality --infer-frames 0 --breakdown-steps 1"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr" -o run -f csv -- python3 bench.py --steps 100 --warmup 5 $Q \
    > "$OUT/b.json" 2> "$OUT/b.err"
for b in 10 11 12; do python3 scripts/timeline.py "$OUT/tr/run_kernel_trace.csv" 20 $b; done > "$OUT/timeline_product.txt"
rm -rf "$OUT/tr"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr8" -o run -f csv -- python3 bench.py --steps 100 --warmup 5 $Q \
    --emulate-dp 8 > "$OUT/b8.json" 2> "$OUT/b8.err"
for b in 10 11; do python3 scripts/timeline.py "$OUT/tr8/run_kernel_trace.csv" 20 $b sample_batch_kernel; done > "$OUT/timeline_emulate_dp8.txt"
rm -rf "$OUT/tr8"
head -8 "$OUT/timeline_product.txt"; head -8 "$OUT/timeline_emulate_dp8.txt"
