# Round 5: split march (gpu_r5y.sh) + the emulated world-8 step re-measured from the single-process trainer's
# state (bench.py --emulate-dp now pretrains world 1 and transplants the state; 300 timed steps).
# usage: gpurun -- bash scripts/gpu_r5z.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5z}
bash scripts/gpu_r5y.sh ${T}y
bash scripts/ab_env.sh ${T}dp 2 "||--steps 300" "||--steps 300 --emulate-dp 8 --dp-fine-buckets 2" \
    "||--steps 300 --emulate-dp 8 --dp-fine-buckets 4"
for f in gpurun_out/${T}dp/v*_*.json; do python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); u=d['roofline']['units_check']
print(sys.argv[1], round(d['value']/1e6,3), d['ms_per_step'], {k: round(v['timed']) for k, v in u.items() if isinstance(v, dict) and 'timed' in v})" $f; done
