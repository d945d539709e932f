# Round 4: where the next batch's march forks off the step, with the row forward (A/B).
# usage: gpurun -- bash scripts/gpu_r4h.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4h2}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 1 $OUT/pytest.log
bash scripts/ab_env.sh ${1:-r4h2}/ab 3 "||" "|NGP_MARCH_AT=start|" "lib_l4r||" "lib_w4r||"
