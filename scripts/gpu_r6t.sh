# Round 6: the update step's period in the driver's 20-step command vs longer windows
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6t; mkdir -p $OUT
F="--no-cpu-baseline --quality-steps 0 --no-oracle-quality --psnr-views 0 --infer-frames 0 --dropin-steps 0"
for st in 20 20 200; do
timeout -k 10 300 python -u bench.py --steps $st --warmup 5 $F > $OUT/b$st.json 2> $OUT/b$st.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], json.dumps(d.get('occupancy_update_step')))" $OUT/b$st.json $st
done
