# Round 5: the training march alone (with / without cell windows) + a dump of its state; then the
# coarse-wide parity tests and A/B (gpu_r5o.sh).
# usage: gpurun -- bash scripts/gpu_r5p.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5p}
mkdir -p gpurun_out/$T
timeout -k 10 240 python -u scripts/diag/march_dump.py > gpurun_out/$T/march_dump.log 2>&1 || { tail -30 gpurun_out/$T/march_dump.log; exit 1; }
tail -1 gpurun_out/$T/march_dump.log
bash scripts/gpu_r5o.sh ${T}o
