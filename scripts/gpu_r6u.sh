# Round 6: occupancy tests (the split update) + trainer tests
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6u; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_occupancy_gpu.py tests/test_trainer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
