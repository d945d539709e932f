set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/swz
for cfg in "NGP_AMD_LIB=build_ab/base.so" "NGP_X=1" "NGP_AMD_LIB=build_ab/base.so" "NGP_X=1"; do
  env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --psnr-views 0 --quality-steps 0 --infer-frames 0 --breakdown-steps 100 > gpurun_out/swz/one.json 2> gpurun_out/swz/one.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/swz/one.json')); k=d['kernels']; print(sys.argv[1], d['value'], k['mlp_bwd']['ms_per_step'], k['hash_encode']['ms_per_step'])" "$cfg" >> gpurun_out/swz/ab.txt
done
BENCH="python3 bench.py --steps 10 --warmup 2 --psnr-views 0 --no-cpu-baseline --infer-frames 0 --quality-steps 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex field_bwd -d gpurun_out/swz/lds -o run -f csv -- $BENCH > gpurun_out/swz/lds.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/swz/lds 10 > gpurun_out/swz/lds.txt
rm -rf gpurun_out/swz/lds
