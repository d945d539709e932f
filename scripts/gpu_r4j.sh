# Round 4: garden-shaped (BASELINE config 4 shape) bench with the round-4 defaults (row forward, march after round 1)
# against the round-3 forward schedule (NGP_ROW_FWD=0 NGP_MARCH_AT=start), alternating.  usage: gpurun -- bash scripts/gpu_r4j.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4q}; mkdir -p $OUT
for rep in 1 2; do
  i=0
  for envs in "" "NGP_ROW_FWD=0"; do
    i=$((i+1))
    env $envs timeout -k 10 300 python -u bench.py --scale 16 --batch 16384 --steps 300 --warmup 10 --no-cpu-baseline \
        --quality-steps 0 --psnr-views 0 --infer-frames 0 --no-oracle-quality --breakdown-steps 20 > "$OUT/v${i}_$rep.json" 2> "$OUT/v${i}_$rep.err"
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']
print('v'+sys.argv[2], sys.argv[3], round(d['value']/1e6,3), 'M rays/s', round(d['ms_per_step']*1e3,1), 'us/step', c.get('rm_samples_per_ray'), c.get('vr_samples_per_ray'), c.get('field_evaluated_per_ray'))" "$OUT/v${i}_$rep.json" "$i" "[$envs]"
  done
done
