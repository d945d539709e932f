# Round 5: the GPU suite and smoke on the final build (the libraries in the tree as shipped).
# usage: gpurun -- bash scripts/gpu_r5pp.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5pp}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$T/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
tail -1 gpurun_out/$T/smoke.log
