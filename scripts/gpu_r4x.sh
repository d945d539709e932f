# Round 4: the forward kernels with 16-wave workgroups (one weight image per CU) vs 8 (A/B).  usage: gpurun -- bash scripts/gpu_r4x.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
NGP_AMD_LIB=$PWD/ar-nerf_amd/lib_w16/libngp_amd.so timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w16_pytest.log 2>&1
tail -n 1 gpurun_out/w16_pytest.log
bash scripts/ab_env.sh ${1:-r4w16}/ab 3 "||" "lib_w16||"
