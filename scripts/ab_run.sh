set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pair
NGP_PAIR_STEPS=1 timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py tests/test_train_scene_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pair/pytest.log 2>&1
bash scripts/gpu_abn.sh ab_pair 3 "NGP_PAIR_STEPS=0" "NGP_PAIR_STEPS=1"
