# Round 5: where the coarse levels' backward + the MLP/coarse Adam run (NGP_COARSE_ORDER).
# usage: gpurun -- bash scripts/gpu_r5j.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5j}
mkdir -p gpurun_out/$T
bash scripts/ab_env.sh $T/ab 2 "||--steps 300" "|NGP_COARSE_ORDER=before|--steps 300" \
    "|NGP_COARSE_ORDER=between|--steps 300" "|NGP_COARSE_ORDER=adam_side|--steps 300"
for f in gpurun_out/$T/ab/v*_1.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value']); [print(f'  {k:18s} {v[0]:7.1f} {v[1]:7.1f}') for k, v in d['probe_timeline_us'].items()]" $f
done
