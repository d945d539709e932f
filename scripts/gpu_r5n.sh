# Round 5: cell windows in the training march (NGP_MARCH_CELLS=1): bit-exact tests, then A/B.
# usage: gpurun -- bash scripts/gpu_r5n.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5n}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_vren_gpu.py -k "march" > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -3
bash scripts/ab_env.sh $T/ab 2 "||--steps 600" "|NGP_MARCH_CELLS=1|--steps 600"
