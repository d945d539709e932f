# Round 4: the compositing kernel's grid capped (NGP_COMPOSITE_BLOCKS; blocks stride over the rows) beside the
# march (A/B; composite tests first).  usage: gpurun -- bash scripts/gpu_r4o.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4w}; mkdir -p $OUT
NGP_COMPOSITE_BLOCKS=64 timeout -k 10 300 python -u -m pytest tests/test_composite_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 1 $OUT/pytest.log
bash scripts/ab_env.sh ${1:-r4w}/ab 3 "||" "|NGP_COMPOSITE_BLOCKS=1024|" "|NGP_COMPOSITE_BLOCKS=512|"
