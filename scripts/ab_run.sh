set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/split
timeout -k 10 400 python -u -m pytest tests/test_trainer_gpu.py tests/test_field_gpu.py -x -v --timeout 120 --timeout-method thread -k "two_part or fused_adam or replicated or binned" > gpurun_out/split/pytest.log 2>&1
NGP_AMD_LIB=build_ab/b12.so timeout -k 10 400 python -u -m pytest tests/test_trainer_gpu.py tests/test_field_gpu.py -x -v --timeout 120 --timeout-method thread -k "fused_adam or binned" > gpurun_out/split/pytest_b12.log 2>&1
bash scripts/gpu_abn.sh ab_split 3 "NGP_BWD_SPLIT=0" "NGP_BWD_SPLIT=128" "NGP_AMD_LIB=build_ab/b12.so" "NGP_BWD_SPLIT=128 NGP_AMD_LIB=build_ab/b12.so"
