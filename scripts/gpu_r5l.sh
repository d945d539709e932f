# Round 5: critical-path cost of the side branches (scripts/diag/skip_cost.py) + the march alone.
# usage: gpurun -- bash scripts/gpu_r5l.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5l}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u scripts/diag/skip_cost.py 300 3 > gpurun_out/$T/skip_cost.log 2>&1 || { tail -30 gpurun_out/$T/skip_cost.log; exit 1; }
tail -14 gpurun_out/$T/skip_cost.log
