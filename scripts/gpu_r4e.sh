# Round 4 check: full GPU suite, smoke, the driver's bench command, a rocprofv3 kernel-stats run,
# then the product and emulated world-8 timelines.  usage: gpurun -- bash scripts/gpu_r4e.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
bash scripts/round_check.sh ${1:-r4e}
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${1:-r4e}/bench_driver_cmd.json 2> gpurun_out/${1:-r4e}/bench_driver_cmd.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('driver cmd', d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['roofline']['units_check']))" gpurun_out/${1:-r4e}/bench_driver_cmd.json
bash scripts/gpu_r4c.sh ${1:-r4e}/tl
