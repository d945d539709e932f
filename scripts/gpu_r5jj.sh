# Round 5: the pre-encode as (row, level pair) wave items -- one gather round per wave instead of four per row
# (r5ii timeline: ~2.7 K row-waves of ~16 us each, 18-27 us past the Adam) -- against the row-per-wave form
# (lib_oldpre); the pre-encode's GPU tests first.
# usage: gpurun -- bash scripts/gpu_r5jj.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5jj}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_field_gpu.py tests/test_trainer_gpu.py -m gpu -k "preencode" > gpurun_out/$T/pytest_pre.log 2>&1 || { tail -40 gpurun_out/$T/pytest_pre.log; exit 1; }
tail -3 gpurun_out/$T/pytest_pre.log
bash scripts/ab_env.sh $T 5 "lib_oldpre||--steps 600" "||--steps 600"
bash scripts/gpu_r5tl.sh ${T}_tl
