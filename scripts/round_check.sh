# Round check on one MI355X: the full GPU suite, smoke, the default bench command (the driver's), a
# rocprofv3 kernel-stats run of a short bench.  usage: gpurun -- bash scripts/round_check.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-rc}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -1 $OUT/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d.get('quality_vs_fp32_oracle')), json.dumps(d.get('inference'))[:300])" $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -f csv -- python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 --infer-frames 0 --no-oracle-quality > $OUT/prof_bench.json 2> $OUT/prof_bench.err
python3 scripts/kstats.py $(find $OUT/prof -name 'run_kernel_trace.csv' | head -1) 200 > $OUT/kstats.txt 2>&1 || true
cp $(find $OUT/prof -name 'run_kernel_stats.csv' | head -1) $OUT/rocprof_kernel_stats.csv || true
python3 scripts/timeline.py $(find $OUT/prof -name 'run_kernel_trace.csv' | head -1) 20 10 > $OUT/timeline.txt 2>&1 || true
rm -rf $OUT/prof
