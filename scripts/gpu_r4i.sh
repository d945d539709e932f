# Round 4: queue priorities for the step's streams (A/B).  usage: gpurun -- bash scripts/gpu_r4i.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4p}; mkdir -p $OUT
timeout -k 10 60 python -c "import torch; print('priority range', torch.cuda.Stream.priority_range(), torch.cuda.Stream(priority=-1).priority)"
bash scripts/ab_env.sh ${1:-r4p}/ab 3 "||" "|NGP_MAIN_PRIO=high|" "|NGP_MAIN_PRIO=high NGP_BWD_PRIO=high|"
