# Round 6: the slot-layout march (ngp_march_train_direct) -- the whole GPU suite, smoke, skip_cost, and
# alternating bench windows against the dense layout (--dense-march).
# usage: gpurun --timeout 1200 -- bash scripts/gpu_r6f.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r6f}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_trainer.log 2>&1 || { tail -60 $OUT/pytest_trainer.log; exit 1; }
tail -1 $OUT/pytest_trainer.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u scripts/diag/skip_cost.py 300 2 full,nomarch > $OUT/skip.txt 2> $OUT/skip.err
tail -1 $OUT/skip.txt
bash scripts/ab_lib.sh $T/ab 3 "::" "::--dense-march"
