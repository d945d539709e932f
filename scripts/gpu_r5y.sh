# Round 5: the next batch's march in two parts (NGP_MARCH_SPLIT=f: rays [0, fR) beside round 2 + composite,
# the rest beside the MLP backward) -- the per-wave timeline showed the composite waiting for slots beside it.
# usage: gpurun -- bash scripts/gpu_r5y.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5y}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_trainer_gpu.py -k "split or prefetched or device_batches" > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
bash scripts/ab_env.sh $T/ab 2 "||--steps 600" "|NGP_MARCH_SPLIT=0.5|--steps 600" "|NGP_MARCH_SPLIT=0.35|--steps 600" "|NGP_MARCH_SPLIT=0.65|--steps 600"
