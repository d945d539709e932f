# Round 5: coarse merge window NG groups x LPW levels per wave (NGP_COARSE_WIDE / NGP_COARSE_LPW): parity, A/B.
# usage: gpurun -- bash scripts/gpu_r5s.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5s}
mkdir -p gpurun_out/$T
for v in "4 2" "8 2" "8 1" "16 2"; do
set -- $v
NGP_COARSE_WIDE=$1 NGP_COARSE_LPW=$2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_field_gpu.py -k "coarse_scatter or levels_replicated or binned_matches" > gpurun_out/$T/pytest_w$1_$2.log 2>&1 || { tail -40 gpurun_out/$T/pytest_w$1_$2.log; exit 1; }
echo "w$1 lpw$2: $(tail -1 gpurun_out/$T/pytest_w$1_$2.log)"
done
bash scripts/ab_env.sh $T/ab 2 "||--steps 600" "|NGP_COARSE_WIDE=4 NGP_COARSE_LPW=2|--steps 600" "|NGP_COARSE_WIDE=8 NGP_COARSE_LPW=2|--steps 600" \
    "|NGP_COARSE_WIDE=8 NGP_COARSE_LPW=1|--steps 600" "|NGP_COARSE_WIDE=16 NGP_COARSE_LPW=2|--steps 600"
