# Round 5: per-wave timeline of the step (scripts/diag/wave_timeline.py, device probes) on the current tree.
# usage: gpurun -- bash scripts/gpu_r5tl.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5tl}
mkdir -p gpurun_out/$T
timeout -k 10 240 python -u scripts/diag/wave_timeline.py 3 > gpurun_out/$T/wave_timeline.log 2>&1 || { tail -30 gpurun_out/$T/wave_timeline.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/wave_timeline.log > gpurun_out/$T/wave_timeline.txt
cut -c1-160 gpurun_out/$T/wave_timeline.txt
mv gpurun_out/wave_timeline.json gpurun_out/$T/
