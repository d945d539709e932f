# Alternating A/B of a modified source file against an alternate copy on the GPU box's scratch tree:
# gpurun -- bash scripts/ab_swap.sh TAG REPS DEST ALT   (A = the tree's DEST, B = ALT copied over DEST)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; REPS=$2; DEST=$3; ALT=$4
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cp "$DEST" "$OUT/A.src"
trap 'cp "$OUT/A.src" "$DEST"' EXIT  # the tree's source is restored however the loop ends
for rep in $(seq 1 $REPS); do
  for v in A B; do
    if [ $v = A ]; then cp "$OUT/A.src" "$DEST"; else cp "$ALT" "$DEST"; fi
    timeout -k 10 200 python -u bench.py --steps 1000 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 \
        --infer-frames 0 --breakdown-steps 20 > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,3), 'M rays/s', round(d['ms_per_step']*1e3,1), 'us/step')" "$OUT/${v}_$rep.json" "$v"
  done
done
