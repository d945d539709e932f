# Round 4: the bucket plan captured after the MLP backward (queue assignment), and the compositing kernel at wave
# priority 2 (A/B, with the trainer tests first).  usage: gpurun -- bash scripts/gpu_r4l.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4t}; mkdir -p $OUT
NGP_PLAN_AFTER=1 timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 1 $OUT/pytest.log
bash scripts/ab_env.sh ${1:-r4t}/ab 3 "||" "|NGP_PLAN_AFTER=1|" "lib_cp||"
