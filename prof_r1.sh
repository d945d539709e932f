set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -f csv -- python3 bench.py --steps 100 --warmup 5 --pretrain 2000 --psnr-views 0 --no-cpu-baseline > gpurun_out/prof/bench_trace.json 2> gpurun_out/prof/bench_trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "field_fwd|hash_bwd|field_bwd|march|composite|adam" -d gpurun_out/prof/pmc_fetch -o run -f csv -- python3 bench.py --steps 20 --warmup 2 --pretrain 2000 --psnr-views 0 --no-cpu-baseline > gpurun_out/prof/bench_fetch.json 2> gpurun_out/prof/bench_fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "field_fwd|hash_bwd|field_bwd|march|composite|adam" -d gpurun_out/prof/pmc_write -o run -f csv -- python3 bench.py --steps 20 --warmup 2 --pretrain 2000 --psnr-views 0 --no-cpu-baseline > gpurun_out/prof/bench_write.json 2> gpurun_out/prof/bench_write.err
timeout -k 10 600 python3 bench.py --steps 300 --warmup 20 > gpurun_out/prof/bench_full.json 2> gpurun_out/prof/bench_full.err
