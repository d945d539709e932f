# A/B of the hash-backward split: coarse/fine overlap on/off x first binned level.
# Usage: gpurun -- bash scripts/ab_hashbwd.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-hb}
mkdir -p "$OUT"
for ov in 1 0; do
  for lo in 8 6 4 0; do
    NGP_BWD_OVERLAP=$ov timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --breakdown-steps 50 --bin-level-lo $lo > "$OUT/ov${ov}_lo${lo}.json" 2> "$OUT/ov${ov}_lo${lo}.err"
    python3 -c "import json;d=json.load(open('$OUT/ov${ov}_lo${lo}.json'));k=d['kernels'];print('overlap $ov lo $lo', d['value'], d['ms_per_step'], {n: k[n]['ms_per_step'] for n in ('hash_bwd_coarse','hash_write','hash_accum') if n in k})"
  done
done
