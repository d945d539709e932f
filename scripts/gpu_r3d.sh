set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3d
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_vren_gpu.py tests/test_composite_gpu.py -k "chunk_segments or ray_segments or composite" > gpurun_out/r3d/t1.log 2>&1
tail -2 gpurun_out/r3d/t1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_trainer_gpu.py tests/test_golden_gpu.py > gpurun_out/r3d/t2.log 2>&1
tail -2 gpurun_out/r3d/t2.log
bash scripts/ab_swap.sh chunkseg 4 ar-nerf_amd/trainer.py scripts/ab_alt/trainer.py
