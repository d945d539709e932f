# Round 4: round 1 of the row forward with each row's first chunk split over a pair of waves (NGP_ROW_SPLIT=1):
# its tests, then an A/B against the default.  usage: gpurun -- bash scripts/gpu_r4t.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4split}; mkdir -p $OUT
NGP_ROW_SPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_field_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 1 $OUT/pytest.log
bash scripts/ab_env.sh ${1:-r4split}/ab 3 "||" "|NGP_ROW_SPLIT=1|"
