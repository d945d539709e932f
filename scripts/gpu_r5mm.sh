# Round 5: the spread of the driver's 20-step window on the final tree -- 8 fresh processes of
# `bench.py --steps 20 --warmup 5` (the driver's timed window; the line's extra blocks skipped), value and the
# window's composited samples per step.
# usage: gpurun -- bash scripts/gpu_r5mm.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5mm}
mkdir -p gpurun_out/$T
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --quality-steps 0 --psnr-views 0 \
      --infer-frames 0 --dropin-steps 0 --no-oracle-quality > gpurun_out/$T/w$i.json 2> gpurun_out/$T/w$i.err
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); u=d['roofline']['units_check']
print('w'+sys.argv[2], round(d['value']/1e6,3), 'M rays/s', round(d['ms_per_step']*1e3,1), 'us/step', 'composited/step', u['composited_per_step']['timed'])" gpurun_out/$T/w$i.json $i
done
