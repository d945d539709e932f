# Round 5 (VERDICT r04 Next #4): the MLP backward's inner-layer exponents from per-block weight bounds
# (lib_bb, -DNGP_BWD_BOUND=1) instead of per-sample maxima: backward parity + quality tests on that build,
# a PMC pass (VALU per MFMA) of each build, then the A/B.
# usage: gpurun -- bash scripts/gpu_r5w.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5w}
mkdir -p gpurun_out/$T
NGP_AMD_LIB=$PWD/ar-nerf_amd/lib_bb/libngp_amd.so timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_field_gpu.py tests/test_quality_gpu.py -k "backward or quality or grad" > gpurun_out/$T/pytest_bb.log 2>&1 || { tail -40 gpurun_out/$T/pytest_bb.log; exit 1; }
grep -E "passed|failed|relative|rel|dB" gpurun_out/$T/pytest_bb.log | tail -12
for v in base bb; do
  LIB=$PWD/ar-nerf_amd/lib/libngp_amd.so; [ $v = bb ] && LIB=$PWD/ar-nerf_amd/lib_bb/libngp_amd.so
  NGP_AMD_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-include-regex field_bwd_mlp -d gpurun_out/$T/pmc_$v -o run -f csv -- python3 bench.py --steps 10 --warmup 2 --psnr-views 0 --no-cpu-baseline --infer-frames 0 --quality-steps 0 --no-oracle-quality --dropin-steps 0 --pretrain 300 --breakdown-steps 4 > gpurun_out/$T/pmc_$v.log 2>&1
  python3 scripts/pmc_summary.py gpurun_out/$T/pmc_$v 10 > gpurun_out/$T/pmc_$v.txt; rm -rf gpurun_out/$T/pmc_$v
  echo "== $v"; cat gpurun_out/$T/pmc_$v.txt
done
bash scripts/ab_env.sh $T/ab 3 "||--steps 600" "lib_bb||--steps 600"
