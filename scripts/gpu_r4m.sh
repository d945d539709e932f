# Round 4: the next batch's march forked from an event recorded after round 1 with round 2 captured first
# (NGP_R1_EVENT=1: round 2 keeps round 1's queue), A/B with the trainer tests first.  usage: gpurun -- bash scripts/gpu_r4m.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4u}; mkdir -p $OUT
NGP_R1_EVENT=1 timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 1 $OUT/pytest.log
bash scripts/ab_env.sh ${1:-r4u}/ab 3 "||" "|NGP_R1_EVENT=1|"
