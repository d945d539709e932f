# Round 5, first box: active-sample dump (coarse-atomics analysis), GPU suite, the driver's bench command
# (with the new probe-based roofline and the drop-in block), and a rocprofv3 kernel trace of a bench run
# whose roofline window the trace markers bracket -> scripts/roofline_check.py.
# usage: gpurun -- bash scripts/gpu_r5a.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5a}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 240 python -u scripts/diag/active_dump.py > $OUT/dump.log 2>&1
tail -1 $OUT/dump.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -1 $OUT/pytest_gpu.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quality-steps 0 --no-oracle-quality > $OUT/bench_driver.json 2> $OUT/bench_driver.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('driver', d['value'], d['ms_per_step'], d['roofline']['op'], d['roofline']['frac'], {k: v['frac'] for k, v in d['ops'].items()}, json.dumps(d.get('dropin')))" $OUT/bench_driver.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -f csv -- python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 --infer-frames 0 --no-oracle-quality --dropin-steps 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
python3 scripts/roofline_check.py $(find $OUT/prof -name 'run_kernel_trace.csv' | head -1) $OUT/prof_bench.json $OUT/kstats_window.txt > $OUT/roofline_check.txt 2>&1 || true
cat $OUT/roofline_check.txt
python3 scripts/kstats.py $(find $OUT/prof -name 'run_kernel_trace.csv' | head -1) 200 > $OUT/kstats.txt 2>&1 || true
python3 scripts/timeline.py $(find $OUT/prof -name 'run_kernel_trace.csv' | head -1) 20 10 > $OUT/timeline.txt 2>&1 || true
rm -rf $OUT/prof
