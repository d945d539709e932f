# Round 6 (third session): the MLP backward against the fp16-storage model of the oracle (test, printed
# errors); the accumulation capped at 80 VGPRs (waves_per_eu 6, 12 spills) vs the tree (93).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ad
timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py -x -v -s --timeout 120 --timeout-method thread -k "fp16_storage_model or backward_parity" > gpurun_out/r6ad/pytest_fp16model.log 2>&1 || true
timeout -k 10 500 bash scripts/ab_lib.sh r6ad 2 "::" "lib_w6::" > gpurun_out/r6ad/ab.txt 2>&1
