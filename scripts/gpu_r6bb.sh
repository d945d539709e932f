# Round 6: the MLP backward's final weight-gradient adds with static accumulator indices (unrolled, rotated start kept):
# field backward tests, the instruction mix (SQ pass) of both builds, alternating 1000-step windows
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6bb; mkdir -p $OUT
NGP_AMD_LIB=$PWD/ar-nerf_amd/lib_atom/libngp_amd.so timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py tests/test_quality_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/pmc_bench.sh 'field_bwd_mlp' r6bb_base "sqw"
NGP_AMD_LIB=$PWD/ar-nerf_amd/lib_atom/libngp_amd.so bash scripts/pmc_bench.sh 'field_bwd_mlp' r6bb_atom "sqw"
cat gpurun_out/pmc_r6bb_base/sqw.txt gpurun_out/pmc_r6bb_atom/sqw.txt
bash scripts/ab_env.sh r6bb 3 "||" "lib_atom||"
