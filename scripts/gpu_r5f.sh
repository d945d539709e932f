# Round 5: where the next batch's march forks (r1 default / fwd / mlp) with and without the pre-encoded
# round 1, two alternating rounds.  usage: gpurun -- bash scripts/gpu_r5f.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5f}
bash scripts/ab_env.sh $T/ab 2 "|NGP_PRE_COARSE=0|--steps 300" "|NGP_PRE_COARSE=1|--steps 300" \
    "|NGP_MARCH_AT=mlp NGP_PRE_COARSE=0|--steps 300" "|NGP_MARCH_AT=mlp NGP_PRE_COARSE=1|--steps 300" \
    "|NGP_MARCH_AT=fwd NGP_PRE_COARSE=0|--steps 300"
for f in gpurun_out/$T/ab/v*_1.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value']); [print(f'  {k:18s} {v[0]:7.1f} {v[1]:7.1f}') for k, v in d['probe_timeline_us'].items()]" $f
done
