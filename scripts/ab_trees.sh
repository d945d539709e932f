# Alternating A/B of whole source trees (a git worktree of an earlier commit, built in place, next to this one):
# configs "TREE|ENV|FLAGS" (TREE "." = this tree), one bench line per run.
# usage: gpurun -- bash scripts/ab_trees.sh TAG REPS ".||" "abtree_r4||" ...
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; REPS=$2; shift 2
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
for rep in $(seq 1 $REPS); do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    tree=$(echo "$cfg" | cut -d'|' -f1); envs=$(echo "$cfg" | cut -d'|' -f2); flags=$(echo "$cfg" | cut -d'|' -f3)
    (cd "$tree" && env $envs timeout -k 10 240 python -u bench.py --steps 600 --warmup 10 --no-cpu-baseline \
        --quality-steps 0 --no-oracle-quality --psnr-views 0 --infer-frames 0 --breakdown-steps 20 $flags \
        > "$OUT/v${i}_$rep.json" 2> "$OUT/v${i}_$rep.err")
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); u=d['roofline'].get('units_check',{})
print('v'+sys.argv[2], sys.argv[3], round(d['value']/1e6,3), 'M rays/s', round(d['ms_per_step']*1e3,1), 'us/step', 'composited/step', round(u.get('composited_per_step',{}).get('timed',0)), 'evaluated/step', round(u.get('evaluated_per_step',{}).get('timed',0)))" "$OUT/v${i}_$rep.json" "$i" "[$cfg]"
  done
done
