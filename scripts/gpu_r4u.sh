# Round 4: spread of the bench's 20-step timed window (the driver's K/W) against the 800-step default, same tree,
# one box (the quality / CPU-baseline / render extras off; the timed steps are the same).  usage: gpurun -- bash scripts/gpu_r4u.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4spread}; mkdir -p $OUT
X="--no-cpu-baseline --no-oracle-quality --quality-steps 0 --infer-frames 0 --psnr-views 0"
for i in 1 2 3 4 5 6; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 $X > $OUT/k20_$i.json 2> $OUT/k20_$i.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); u=d['roofline']['units_check']; print('K=20', d['value'], d['ms_per_step'], u['composited_per_step']['timed'])" $OUT/k20_$i.json
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 800 --warmup 10 $X > $OUT/k800_$i.json 2> $OUT/k800_$i.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); u=d['roofline']['units_check']; print('K=800', d['value'], d['ms_per_step'], u['composited_per_step']['timed'])" $OUT/k800_$i.json
done
