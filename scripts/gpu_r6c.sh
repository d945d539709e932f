# Round 6: API composite kernels (wave per ray) vs the serial ones bit for bit; march variants on one batch;
# the drop-in path after the sparse backward / composite / get_rays changes.
# usage: gpurun --timeout 900 -- bash scripts/gpu_r6c.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r6c}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 120 python -u scripts/diag/composite_libs.py ar-nerf_amd/lib_base/libngp_amd.so ar-nerf_amd/lib/libngp_amd.so > $OUT/composite_libs.json 2> $OUT/composite_libs.err || { tail -20 $OUT/composite_libs.err; exit 1; }
cat $OUT/composite_libs.json
timeout -k 10 300 python -u scripts/diag/march_libs.py 1500 ar-nerf_amd/lib_base/libngp_amd.so ar-nerf_amd/lib/libngp_amd.so ar-nerf_amd/lib_m7/libngp_amd.so ar-nerf_amd/lib_dbl/libngp_amd.so ar-nerf_amd/lib_dbl7/libngp_amd.so > $OUT/march_libs.txt 2> $OUT/march_libs.err || { tail -20 $OUT/march_libs.err; exit 1; }
cat $OUT/march_libs.txt
timeout -k 10 400 python -u -m pytest tests/test_vren_gpu.py tests/test_field_gpu.py tests/test_dropin_gpu.py tests/test_golden_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u scripts/diag/dropin_profile.py 2000 40 > $OUT/dropin.json 2> $OUT/dropin.err
cat $OUT/dropin.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dprof -o run -f csv -- python3 scripts/diag/dropin_profile.py 2000 40 > $OUT/dropin_prof.json 2> $OUT/dropin_prof.err
TR=$(find $OUT/dprof -name 'run_kernel_trace.csv' | head -1)
python3 scripts/kstats.py $TR 40 > $OUT/dropin_kstats.txt 2>&1 || true
head -24 $OUT/dropin_kstats.txt
rm -rf $OUT/dprof
