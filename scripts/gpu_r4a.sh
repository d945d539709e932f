# Round 4 check: the list / counter tests, then two short benches (the driver's window and a long one)
# with the per-window unit check.  usage: gpurun -- bash scripts/gpu_r4a.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4a}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_vren_gpu.py tests/test_trainer_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 1 $OUT/pytest.log
Q="--no-cpu-baseline --quality-steps 0 --psnr-views 0 --infer-frames 0 --no-oracle-quality"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $Q > $OUT/bench20.json 2> $OUT/bench20.err
timeout -k 10 300 python -u bench.py --steps 800 $Q > $OUT/bench800.json 2> $OUT/bench800.err
for f in bench20 bench800; do
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['frac'], r['ms_per_step'], json.dumps(r['units_check']))" $OUT/$f.json
done
