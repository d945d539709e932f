# Round 6: the new guard / RCCL-occupancy tests first, then the whole GPU suite, smoke and the driver's bench command.
# usage: gpurun --timeout 1100 -- bash scripts/gpu_r6a.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r6a}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_guard_gpu.py tests/test_ddp_gpu.py -k "guard or overflow or rccl" -x -v --timeout 200 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -80 $OUT/pytest_new.log; exit 1; }
tail -3 $OUT/pytest_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('driver cmd', d['value'], d['ms_per_step'], d['ns_per_composited_sample'], d['guard_hits'], d['roofline']['op'], d['roofline']['frac'], d['probe_step_gaps_us'], json.dumps(d.get('dropin'))[:200], json.dumps(d.get('quality'))[:300])" $OUT/bench_driver_cmd.json
