# Round 6: the occupancy update's parameter-independent head beside the step before it; GPU suite + bench lines
# (occupancy_update_step) on 1000-step windows.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6r}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
F="--no-cpu-baseline --quality-steps 0 --no-oracle-quality --psnr-views 0 --infer-frames 0 --dropin-steps 0"
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 10 $F > $OUT/b$i.json 2> $OUT/b$i.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['ns_per_composited_sample'], json.dumps(d.get('occupancy_update_step')))" $OUT/b$i.json
done
