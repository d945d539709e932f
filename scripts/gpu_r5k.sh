# Round 5: the occupancy update evaluating only the samples it keeps (NGP_OCC_KEEP).
# usage: gpurun -- bash scripts/gpu_r5k.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5k}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_occupancy_gpu.py \
    tests/test_vren_gpu.py -k "keep or occupancy or update" > gpurun_out/$T/pytest.log 2>&1 \
    || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
grep -E "passed|failed|kept" gpurun_out/$T/pytest.log | tail -5
bash scripts/ab_env.sh $T/ab 3 "|NGP_OCC_KEEP=0|--steps 400" "||--steps 400"
