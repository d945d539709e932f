# Round 5: per-wave march spans (march_dump.py) + coarse merge window 4 vs 8 groups (parity + A/B).
# usage: gpurun -- bash scripts/gpu_r5q.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5q}
mkdir -p gpurun_out/$T
timeout -k 10 240 python -u scripts/diag/march_dump.py > gpurun_out/$T/march_dump.log 2>&1 || { tail -30 gpurun_out/$T/march_dump.log; exit 1; }
tail -1 gpurun_out/$T/march_dump.log
NGP_COARSE_WIDE=8 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_field_gpu.py -k "coarse_scatter or levels_replicated or binned_matches" > gpurun_out/$T/pytest_w8.log 2>&1 || { tail -40 gpurun_out/$T/pytest_w8.log; exit 1; }
grep -E "passed|failed" gpurun_out/$T/pytest_w8.log | tail -2
bash scripts/ab_env.sh $T/ab 2 "||--steps 600" "|NGP_COARSE_WIDE=4|--steps 600" "|NGP_COARSE_WIDE=8|--steps 600"
