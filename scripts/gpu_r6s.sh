# Round 6: kernel trace of a bench run (the occupancy update's kernels: pre-encoded density forward)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6s; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -f csv -- python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 --infer-frames 0 --no-oracle-quality --dropin-steps 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
TR=$(find $OUT/prof -name 'run_kernel_trace.csv' | head -1)
python3 scripts/kstats.py $TR 200 > $OUT/kstats.txt 2>&1 || true
rm -rf $OUT/prof
grep -i "encode\|occ_\|grid_ema\|scatter_kept\|packbits\|zero_words" $OUT/kstats.txt | cut -c1-160
