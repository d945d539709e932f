# Round 6 (third session): the MLP backward at 12 waves per block (3 per SIMD, 147 VGPRs; v2, lib_cw12) vs 8 (v1,
# the tree); its parity tests first on the variant.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ai
NGP_AMD_LIB=$PWD/ar-nerf_amd/lib_cw12/libngp_amd.so timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread -k "backward or training_step" > gpurun_out/r6ai/pytest_cw12.log 2>&1
timeout -k 10 800 bash scripts/ab_lib.sh r6ai 4 "::" "lib_cw12::" > gpurun_out/r6ai/ab.txt 2>&1
