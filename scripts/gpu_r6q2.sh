# Round 6: the occupancy update step's cost (bench line's occupancy_update_step) single-process and in the
# emulated world-8 data-parallel step; the garden-shaped configuration on the round-6 tree.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6q2; mkdir -p $OUT
F="--no-cpu-baseline --quality-steps 0 --no-oracle-quality --psnr-views 0 --infer-frames 0 --dropin-steps 0"
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 $F > $OUT/b1.json 2> $OUT/b1.err
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 $F --emulate-dp 8 > $OUT/b8.json 2> $OUT/b8.err
for f in b1 b8; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['config']['parallelism'][:60], json.dumps(d.get('occupancy_update_step')))" $OUT/$f.json; done
timeout -k 10 300 python -u bench.py --scale 16 --batch 16384 --steps 300 --warmup 10 $F > $OUT/garden.json 2> $OUT/garden.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('garden', d['value'], d['ms_per_step'], d.get('guard_hits'), json.dumps(d['roofline'].get('units_check',{}).get('marched_per_step')), json.dumps(d['roofline'].get('units_check',{}).get('composited_per_step')))" $OUT/garden.json
