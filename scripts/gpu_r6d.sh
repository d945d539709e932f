# Round 6: the doubling march (segment in registers, 65 VGPRs: all waves resident) in the step -- tests,
# march variants on one batch, skip_cost, alternating bench windows (lib_base = round-5 march).
# usage: gpurun --timeout 1200 -- bash scripts/gpu_r6d.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r6d}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 120 python -u scripts/diag/composite_libs.py ar-nerf_amd/lib_serial/libngp_amd.so ar-nerf_amd/lib/libngp_amd.so > $OUT/composite_libs.json 2> $OUT/composite_libs.err || { tail -20 $OUT/composite_libs.err; exit 1; }
cat $OUT/composite_libs.json
timeout -k 10 400 python -u -m pytest tests/test_vren_gpu.py tests/test_field_gpu.py tests/test_dropin_gpu.py tests/test_golden_gpu.py tests/test_renderer_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u scripts/diag/march_libs.py 1500 ar-nerf_amd/lib_base/libngp_amd.so ar-nerf_amd/lib/libngp_amd.so ar-nerf_amd/lib_w8/libngp_amd.so > $OUT/march_libs.txt 2> $OUT/march_libs.err || { tail -20 $OUT/march_libs.err; exit 1; }
cat $OUT/march_libs.txt
for lib in lib_base lib; do
  NGP_AMD_LIB=$PWD/ar-nerf_amd/$lib/libngp_amd.so timeout -k 10 300 python -u scripts/diag/skip_cost.py 300 2 full,nomarch > $OUT/skip_$lib.txt 2> $OUT/skip_$lib.err
  echo $lib; tail -1 $OUT/skip_$lib.txt
done
bash scripts/ab_lib.sh $T/ab 3 "lib_base::" "::" "lib_w8::"
timeout -k 10 300 python -u scripts/diag/dropin_profile.py 2000 40 > $OUT/dropin.json 2> $OUT/dropin.err
cat $OUT/dropin.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dprof -o run -f csv -- python3 scripts/diag/dropin_profile.py 2000 40 > $OUT/dropin_prof.json 2> $OUT/dropin_prof.err
TR=$(find $OUT/dprof -name 'run_kernel_trace.csv' | head -1)
python3 scripts/kstats.py $TR 40 > $OUT/dropin_kstats.txt 2>&1 || true
head -24 $OUT/dropin_kstats.txt
rm -rf $OUT/dprof
