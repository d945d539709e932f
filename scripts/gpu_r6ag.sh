# Round 6 (third session): HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) vs the default;
# the tightened trainer-step gradient bars first.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ag
timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r6ag/pytest_trainer.log 2>&1
timeout -k 10 700 bash scripts/ab_env.sh r6ag 4 "||" "|HIP_FORCE_DEV_KERNARG=1|" > gpurun_out/r6ag/ab.txt 2>&1
