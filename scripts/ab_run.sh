set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fem2 gpurun_out/garden
timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py tests/test_renderer_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fem2/pytest.log 2>&1
bash scripts/gpu_abn.sh ab_fem2 3 "NGP_AMD_LIB=build_ab/base.so" "NGP_X=1"
timeout -k 10 400 python -u bench.py --scale 16 --batch 16384 --no-cpu-baseline --quality-steps 0 --psnr-views 0 > gpurun_out/garden/bench_garden_shaped.json 2> gpurun_out/garden/bench.err
