# DP pipeline tests + product trained state for the glue render + emulated world-N step times
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r3b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ddp_gpu.py > $OUT/ddp.log 2>&1
tail -3 $OUT/ddp.log
timeout -k 10 300 python -u scripts/quality_state.py $OUT/q > $OUT/q.log 2>&1
tail -1 $OUT/q.log
for rep in 1 2; do
for n in 0 1 2 8; do
  timeout -k 10 200 python -u bench.py --steps 1000 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 \
      --infer-frames 0 --breakdown-steps 20 --emulate-dp $n > $OUT/e${n}_$rep.json 2> $OUT/e${n}_$rep.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('emulate', sys.argv[2], round(d['value']/1e6,3), 'M rays/s', round(d['ms_per_step']*1e3,1), 'us/step')" $OUT/e${n}_$rep.json $n
done; done
