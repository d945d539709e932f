# Round 6 (third session): the fused accumulation's Adam flush with its loads issued together.
# v1 = HEAD before the change (lib_base), v2 = the tree (103 VGPRs), v3 = the tree capped at 96 VGPRs,
# v4 / v5 = 3 / 4 records in flight per thread in the record phase (105 / 112 VGPRs).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ac
timeout -k 10 700 bash scripts/ab_lib.sh r6ac 2 "base::" "::" "lib_fg2w5::" "lib_u3::" "lib_u4::" > gpurun_out/r6ac/ab.txt 2>&1
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6ac/pytest_gpu.log 2>&1
