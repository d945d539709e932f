# Round 6: the lattice march rewrite (scalar chain, segment in registers, 64 VGPRs) -- march parity tests on
# the tree's library, then the march alone, the march branch's step cost (skip_cost full vs nomarch) and
# alternating bench windows for lib_base (previous march), lib_m7 (new march, 7 waves/SIMD) and the tree (8).
# usage: gpurun --timeout 1200 -- bash scripts/gpu_r6b.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r6b}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_vren_gpu.py tests/test_golden_gpu.py tests/test_renderer_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_march.log 2>&1 || { tail -60 $OUT/pytest_march.log; exit 1; }
tail -1 $OUT/pytest_march.log
for lib in lib_base lib_m7 lib; do
  NGP_AMD_LIB=$PWD/ar-nerf_amd/$lib/libngp_amd.so timeout -k 10 200 python -u scripts/diag/march_alone.py > $OUT/alone_$lib.json 2> $OUT/alone_$lib.err
  cat $OUT/alone_$lib.json
done
for lib in lib_base lib; do
  NGP_AMD_LIB=$PWD/ar-nerf_amd/$lib/libngp_amd.so timeout -k 10 300 python -u scripts/diag/skip_cost.py 300 2 full,nomarch > $OUT/skip_$lib.txt 2> $OUT/skip_$lib.err
  echo $lib; tail -1 $OUT/skip_$lib.txt
done
bash scripts/ab_lib.sh $T/ab 2 "lib_base::" "lib_m7::" "::"
# the drop-in loop: wall time, host-side op profile, and a rocprofv3 kernel trace of its steps
timeout -k 10 300 python -u scripts/diag/dropin_profile.py 2000 40 --torch-profile > $OUT/dropin.json 2> $OUT/dropin_torchprof.txt
cat $OUT/dropin.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dprof -o run -f csv -- python3 scripts/diag/dropin_profile.py 2000 40 > $OUT/dropin_prof.json 2> $OUT/dropin_prof.err
TR=$(find $OUT/dprof -name 'run_kernel_trace.csv' | head -1)
python3 scripts/kstats.py $TR 40 > $OUT/dropin_kstats.txt 2>&1 || true
head -30 $OUT/dropin_kstats.txt
rm -rf $OUT/dprof
