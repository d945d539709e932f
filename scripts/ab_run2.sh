set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pad2
timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread -k "backward or step or fused" > gpurun_out/pad2/pytest.log 2>&1
BENCH="python3 bench.py --steps 10 --warmup 2 --psnr-views 0 --no-cpu-baseline --infer-frames 0 --quality-steps 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex field_bwd -d gpurun_out/pad2/lds -o run -f csv -- $BENCH > gpurun_out/pad2/lds.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/pad2/lds 10 > gpurun_out/pad2/lds.txt
rm -rf gpurun_out/pad2/lds
