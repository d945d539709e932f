# Round 6: the march with its compaction inside (ngp_march_train_direct, packed layout) -- trainer + march tests,
# skip_cost, alternating bench windows against the separate scan / compaction launches (--dense-march), then the
# 3-seed quality run at the reference schedule.
# usage: gpurun --timeout 1200 -- bash scripts/gpu_r6h.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r6h}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_trainer_gpu.py tests/test_vren_gpu.py tests/test_golden_gpu.py tests/test_guard_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u scripts/diag/skip_cost.py 300 2 full,nomarch > $OUT/skip.txt 2> $OUT/skip.err
tail -1 $OUT/skip.txt
bash scripts/ab_lib.sh $T/ab 3 "::" "::--dense-march"
bash scripts/gpu_r6q.sh ${T}q
