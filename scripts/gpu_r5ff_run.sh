# the pre-encode's GPU tests, then the r5ff A/B (usage: gpurun -- bash scripts/gpu_r5ff_run.sh TAG)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5ff}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_field_gpu.py tests/test_trainer_gpu.py -m gpu -k "preencoded or first or trains_like" > gpurun_out/$T/pytest_pre.log 2>&1 || { tail -40 gpurun_out/$T/pytest_pre.log; exit 1; }
tail -3 gpurun_out/$T/pytest_pre.log
bash scripts/gpu_r5ff.sh $T
