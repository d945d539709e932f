# Round 5: probe timelines of the default step (pre-encode off / on) and the 4096-entry-bucket
# accumulation variant (lib_b12, two accumulating workgroups per CU).  usage: gpurun -- bash scripts/gpu_r5d.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5d}
bash scripts/ab_env.sh $T/ab 2 "|NGP_PRE_COARSE=0|--steps 400" "|NGP_PRE_COARSE=1|--steps 400" "lib_b12|NGP_PRE_COARSE=0|--steps 400"
for f in gpurun_out/$T/ab/v*_1.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1]); [print(f'  {k:18s} {v[0]:7.1f} {v[1]:7.1f}') for k, v in d['probe_timeline_us'].items()]" $f
done
