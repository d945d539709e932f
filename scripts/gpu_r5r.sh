# Round 5: cell windows x march grid cap (NGP_MARCH_BLOCKS: resident march waves beside the step).
# usage: gpurun -- bash scripts/gpu_r5r.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5r}
mkdir -p gpurun_out/$T
bash scripts/ab_env.sh $T/ab 2 "||--steps 600" "|NGP_MARCH_CELLS=1|--steps 600" "|NGP_MARCH_CELLS=1 NGP_MARCH_BLOCKS=1024|--steps 600" \
    "|NGP_MARCH_CELLS=1 NGP_MARCH_BLOCKS=512|--steps 600" "|NGP_MARCH_BLOCKS=512|--steps 600"
