# Round-4 final check on one MI355X: the full GPU suite, smoke, the default bench command, the driver's bench
# command, a rocprofv3 kernel-stats run + timeline, then PMC FETCH_SIZE / WRITE_SIZE passes of the hash backward's
# and the forward's kernels (-> pmc_traffic.json).  usage: gpurun -- bash scripts/gpu_r4_final.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/round_check.sh ${1:-r4z}
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${1:-r4z}/bench_driver_cmd.json 2> gpurun_out/${1:-r4z}/bench_driver_cmd.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('driver cmd', d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['roofline']['units_check']))" gpurun_out/${1:-r4z}/bench_driver_cmd.json
bash scripts/pmc_bench.sh 'hash_write|hash_accum|hash_adam_residual|adam_kernel|field_|hash_bwd_kernel' ${1:-r4z} "fetch write"
python3 scripts/pmc_traffic.py gpurun_out/pmc_${1:-r4z} gpurun_out/${1:-r4z}/pmc_traffic.json > /dev/null
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(k, v['bytes_per_launch'], v.get('dur_us_fetch_pass')) for k, v in d.items() if k[0] != '_']" gpurun_out/${1:-r4z}/pmc_traffic.json
