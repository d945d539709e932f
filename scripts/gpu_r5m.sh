# Round 5: the training march as a lane-per-ray walk (NGP_MARCH_LANE = rays per wave) vs the wave-per-ray
# lattice walk: the march branch costs the step ~its own duration (skip_cost.py), so a light,
# slow walk beside the step may beat a fast, heavy one.
# usage: gpurun -- bash scripts/gpu_r5m.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5m}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_vren_gpu.py > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
bash scripts/ab_env.sh $T/ab 2 "||--steps 600" "|NGP_MARCH_LANE=64|--steps 600" "|NGP_MARCH_LANE=32|--steps 600" "|NGP_MARCH_LANE=16|--steps 600"
