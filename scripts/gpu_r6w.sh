# Round 6: the coarse hash kernel as 256 blocks x 8 waves (one block per CU: 2 waves x 64 VGPRs per SIMD next to
# the accumulation's 4 x 96) instead of 512 x 4 (uneven: CUs with 3-4 coarse waves per SIMD keep the
# accumulation's blocks out); coarse-scatter tests, alternating 1000-step windows
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6w; mkdir -p $OUT
NGP_AMD_LIB=$PWD/ar-nerf_amd/lib_cw8/libngp_amd.so timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "coarse or scatter or binned or backward" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/ab_env.sh r6w 3 "||" "lib_cw8||"
