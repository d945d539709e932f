# Round 6: the compositing kernel with no chunk held across its passes (every chunk's w / Ta parked in memory and
# read back: fewer VGPRs, one more round trip per chunk), uncapped (97 VGPRs) and capped at 64 (8 waves/SIMD,
# 32 spilled) so its waves can start beside the march; composite tests on each, alternating 1000-step windows
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6z; mkdir -p $OUT
for v in cproto cproto8; do
NGP_AMD_LIB=$PWD/ar-nerf_amd/lib_$v/libngp_amd.so timeout -k 10 300 python -u -m pytest tests/test_composite_gpu.py tests/test_distortion_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
echo "$v $(tail -1 $OUT/pytest_$v.log)"
done
bash scripts/ab_env.sh r6z 3 "||" "lib_cproto||" "lib_cproto8||"
