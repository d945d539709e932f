# Round 5: register caps on the composite (lib_c5: 5 waves/SIMD) and the march (lib_m6: 6 waves/SIMD) -- the
# per-wave timeline shows the composite's waves waiting for slots beside the march.
# usage: gpurun -- bash scripts/gpu_r5u.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5u}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_composite_gpu.py tests/test_distortion_gpu.py tests/test_field_gpu.py -k "composite or distortion or outside" > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
bash scripts/ab_env.sh $T/ab 2 "||--steps 600" "lib_c5||--steps 600" "lib_m6||--steps 600" "lib_c5m6||--steps 600" "lib_m6|NGP_MARCH_CELLS=1|--steps 600"
