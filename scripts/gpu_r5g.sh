# Round 5: capture order at the step's forks (critical child first vs side branch first), the
# changed tests first.  usage: gpurun -- bash scripts/gpu_r5g.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5g}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_field_gpu.py \
    tests/test_trainer_gpu.py -k "capture_order or first or coarse or pair or graph" > gpurun_out/$T/pytest.log 2>&1 \
    || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
grep "crit-first" gpurun_out/$T/pytest.log || true
bash scripts/ab_env.sh $T/ab 2 "|NGP_CRIT_FIRST=0|--steps 300" "|NGP_CRIT_FIRST=2|--steps 300" "|NGP_CRIT_FIRST=4|--steps 300" "|NGP_CRIT_FIRST=6|--steps 300"
for f in gpurun_out/$T/ab/v*_1.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d.get('probe_step_gaps_us')); [print(f'  {k:18s} {v[0]:7.1f} {v[1]:7.1f}') for k, v in d['probe_timeline_us'].items()]" $f
done
