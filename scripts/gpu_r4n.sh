# Round 4: the training march's grid capped (NGP_MARCH_BLOCKS: a grid-stride over the rays), so the march beside
# round 2 / the composite / the MLP backward holds fewer CU slots (A/B, march tests first).  usage: gpurun -- bash scripts/gpu_r4n.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4v}; mkdir -p $OUT
NGP_MARCH_BLOCKS=64 timeout -k 10 300 python -u -m pytest tests/test_vren_gpu.py tests/test_golden_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 1 $OUT/pytest.log
bash scripts/ab_env.sh ${1:-r4v}/ab 3 "||" "|NGP_MARCH_BLOCKS=512|" "|NGP_MARCH_BLOCKS=256|"
