# Round 6: drop-in path (block-aggregated gradient rows, replicated coarse levels, zero_grad default) + the
# 8-wave march as the default: parity subset, drop-in wall time + kernel trace, the driver's bench command.
# usage: gpurun --timeout 900 -- bash scripts/gpu_r6e.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r6e}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_vren_gpu.py tests/test_field_gpu.py tests/test_dropin_gpu.py tests/test_golden_gpu.py tests/test_trainer_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u scripts/diag/dropin_profile.py 2000 40 --torch-profile > $OUT/dropin.json 2> $OUT/dropin_torchprof.txt
cat $OUT/dropin.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dprof -o run -f csv -- python3 scripts/diag/dropin_profile.py 2000 40 > $OUT/dropin_prof.json 2> $OUT/dropin_prof.err
TR=$(find $OUT/dprof -name 'run_kernel_trace.csv' | head -1)
python3 scripts/kstats.py $TR 40 > $OUT/dropin_kstats.txt 2>&1 || true
head -16 $OUT/dropin_kstats.txt
rm -rf $OUT/dprof
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('driver cmd', d['value'], d['ms_per_step'], d['ns_per_composited_sample'], d['guard_hits'], d['roofline']['op'], d['roofline']['frac'], 'mlp_fwd', d['ops'].get('mlp_fwd', {}).get('frac'), 'mlp_bwd', d['ops'].get('mlp_bwd', {}).get('frac'), json.dumps(d.get('dropin'))[:120], json.dumps(d.get('inference'))[:160], json.dumps(d.get('quality'))[:200])" $OUT/bench_driver_cmd.json
