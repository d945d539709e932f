# Round 5: coarse hash backward with runs merged across NG 16-sample groups (NGP_COARSE_WIDE=NG):
# parity tests under the knob, then A/B against the 16-sample merge window.
# usage: gpurun -- bash scripts/gpu_r5o.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5o}
mkdir -p gpurun_out/$T
for w in 4 2; do
NGP_COARSE_WIDE=$w timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_field_gpu.py -k "coarse_scatter or levels_replicated or binned_matches" > gpurun_out/$T/pytest_w$w.log 2>&1 || { tail -40 gpurun_out/$T/pytest_w$w.log; exit 1; }
grep -E "passed|failed" gpurun_out/$T/pytest_w$w.log | tail -2
done
bash scripts/ab_env.sh $T/ab 2 "||--steps 600" "|NGP_COARSE_WIDE=4|--steps 600" "|NGP_COARSE_WIDE=2|--steps 600"
