# Round 6 (third session): the MLP backward against the oracle's fp16-storage model (printed errors);
# the GPU suite on the tree; then alternating: v1 = HEAD (lib_base), v2 = the tree (the binned count pass + its scan with
# one (tile, level) item per block iteration), v3 = the tree + the accumulation capped at 80 VGPRs (12 spills).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ae
timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py -x -v -s --timeout 120 --timeout-method thread -k "fp16_storage_model or backward_parity" > gpurun_out/r6ae/pytest_fp16model.log 2>&1 || true
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6ae/pytest_gpu.log 2>&1
timeout -k 10 600 bash scripts/ab_lib.sh r6ae 3 "base::" "::" "lib_w6::" > gpurun_out/r6ae/ab.txt 2>&1
