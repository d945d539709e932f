# Generic alternating A/B of bench flag sets: gpurun -- bash scripts/ab_generic.sh TAG REPS "flagsA" "flagsB" ["flagsC"]
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in $(seq 1 $REPS); do
  i=0
  for flags in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python -u bench.py --steps 1000 --warmup 10 --no-cpu-baseline --quality-steps 0 --no-oracle-quality --psnr-views 0 \
        --infer-frames 0 --breakdown-steps 20 $flags > "$OUT/v${i}_$rep.json" 2> "$OUT/v${i}_$rep.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('v'+sys.argv[2], sys.argv[3], round(d['value']/1e6,3), 'M rays/s', round(d['ms_per_step']*1e3,1), 'us/step')" "$OUT/v${i}_$rep.json" "$i" "[$flags]"
  done
done
