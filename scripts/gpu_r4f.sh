# Round 4: data-parallel step (emulated world 8) with 1 / 2 / 4 fine buckets, and its tests.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4f}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_ddp.log 2>&1
tail -n 1 $OUT/pytest_ddp.log
bash scripts/ab_env.sh ${1:-r4f}/ab 2 "|| --emulate-dp 8 --dp-fine-buckets 1" "|| --emulate-dp 8 --dp-fine-buckets 2" "|| --emulate-dp 8 --dp-fine-buckets 4" "||" "|NGP_FUSED_COARSE=1|" "lib_r3|NGP_FEM_LDS=1|"
timeout -k 10 120 python -u scripts/diag/rccl_host_cost.py > $OUT/rccl_host.json 2> $OUT/rccl_host.err && cat $OUT/rccl_host.json
