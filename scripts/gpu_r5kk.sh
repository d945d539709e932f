# Round 5: where the next batch's march forks, re-measured on the final tree (the pre-encode now runs at any fork
# point): after round 1 (default) vs after round 2 (fwd: the composite would not share the register file with the
# march's first waves) vs at the step's start.
# usage: gpurun -- bash scripts/gpu_r5kk.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5kk}
bash scripts/ab_env.sh $T 5 "||--steps 600" "|NGP_MARCH_AT=fwd|--steps 600" "|NGP_MARCH_AT=start|--steps 600"
