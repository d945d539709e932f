# guard hits of the occupancy-list kernels, default vs exact mode (30k steps each)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xf
python3 -c "import sys; sys.path.insert(0, 'ar-nerf_amd'); import synthetic as S; S.write_nsvf_scene('/tmp/Synthetic_NeRF/Analytic', res=400, n_train=100, n_test=10)"
timeout -k 10 300 python3 -u scripts/train_scene.py --dataset nsvf --root /tmp/Synthetic_NeRF/Analytic --downsample 0.5 --steps 30000 --test-views 2 --exact > gpurun_out/xf/default.json 2> gpurun_out/xf/default.err

