# Round 4: re-check of the final tree: the GPU suite, smoke, the driver's bench command.
# usage: gpurun -- bash scripts/gpu_r4q.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4q2}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 1 $OUT/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; print('driver cmd', d['value'], d['ms_per_step'], c['row_forward'], c['march_fork'], d['roofline']['frac'])" $OUT/bench_driver_cmd.json
