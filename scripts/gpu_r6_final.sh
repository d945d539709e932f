# Round-6 final check on one MI355X: the GPU suite, smoke, the driver's bench command (full line), a rocprofv3
# kernel trace of a bench run (the roofline window's kernel statistics + scripts/roofline_check.py), the PMC
# FETCH_SIZE / WRITE_SIZE / atomic passes (-> pmc_traffic.json), and the per-wave timeline of the step.
# usage: gpurun --timeout 1200 -- bash scripts/gpu_r6_final.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r6final}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests/test_golden_gpu.py tests/test_field_gpu.py -q -s --timeout 120 --timeout-method thread -k "train or backward" > $OUT/pytest_prints.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('driver cmd', d['value'], d['ms_per_step'], d['ns_per_composited_sample'], d['guard_hits'], d['roofline']['op'], d['roofline']['frac'], json.dumps(d.get('dropin'))[:120], json.dumps(d.get('inference'))[:200], json.dumps(d.get('quality'))[:200])" $OUT/bench_driver_cmd.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -f csv -- python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 --infer-frames 0 --no-oracle-quality --dropin-steps 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
TR=$(find $OUT/prof -name 'run_kernel_trace.csv' | head -1)
python3 scripts/roofline_check.py $TR $OUT/prof_bench.json $OUT/kstats_window.txt > $OUT/roofline_check.txt 2>&1 || true
cat $OUT/roofline_check.txt
python3 scripts/kstats.py $TR 200 > $OUT/kstats.txt 2>&1 || true
cp $(find $OUT/prof -name 'run_kernel_stats.csv' | head -1) $OUT/rocprof_kernel_stats.csv || true
rm -rf $OUT/prof
bash scripts/pmc_bench.sh 'hash_write|hash_accum|hash_adam_residual|adam_kernel|field_|encode_coarse|hash_bwd_kernel|march_slots' $T "fetch write atom"
python3 scripts/pmc_traffic.py gpurun_out/pmc_$T $OUT/pmc_traffic.json > /dev/null
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(k, v['bytes_per_launch'], v.get('dur_us_fetch_pass')) for k, v in d.items() if k[0] != '_']" $OUT/pmc_traffic.json
timeout -k 10 300 python -u scripts/diag/wave_timeline.py 4 > $OUT/wave_timeline.txt 2> $OUT/wave_timeline.err || true
head -20 $OUT/wave_timeline.txt
