# Round 5: per-wave timeline of the step (wave_timeline.py) + the march kernel's own cost (skip_cost.py).
# usage: gpurun -- bash scripts/gpu_r5t.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5t}
mkdir -p gpurun_out/$T
timeout -k 10 240 python -u scripts/diag/wave_timeline.py 3 > gpurun_out/$T/wave_timeline.log 2>&1 || { tail -30 gpurun_out/$T/wave_timeline.log; exit 1; }
cat gpurun_out/$T/wave_timeline.log | grep -v amdgpu.ids
mv gpurun_out/wave_timeline.json gpurun_out/$T/
timeout -k 10 400 python -u scripts/diag/skip_cost.py 300 2 full,nomarchkernel,nomarch > gpurun_out/$T/skip_cost.log 2>&1 || { tail -30 gpurun_out/$T/skip_cost.log; exit 1; }
tail -1 gpurun_out/$T/skip_cost.log
