# Round 5: round 1 with 4 levels per gather round (two dependent rounds for levels 8-15 after the pre-encode) in
# 4-wave blocks (default) vs the previous 2 levels per round in 8-wave blocks (lib_r1old) vs 4 levels in 8-wave
# blocks (lib_r1w8); round 1's bit-exactness tests first, the timeline last.
# usage: gpurun -- bash scripts/gpu_r5oo.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5oo}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_field_gpu.py tests/test_trainer_gpu.py -m gpu -k "first or preencode or row_forward or chunk" > gpurun_out/$T/pytest_r1.log 2>&1 || { tail -40 gpurun_out/$T/pytest_r1.log; exit 1; }
tail -3 gpurun_out/$T/pytest_r1.log
bash scripts/ab_env.sh $T 5 "||--steps 600" "lib_r1old||--steps 600" "lib_r1w8||--steps 600"
bash scripts/gpu_r5tl.sh ${T}_tl
