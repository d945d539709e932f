set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/gc
timeout -k 10 200 python -u scripts/quality_grad_check.py gpu qstate > gpurun_out/gc/gc.log 2>&1
cp qstate/grad_gpu.pt gpurun_out/gc/
tail -1 gpurun_out/gc/gc.log
bash scripts/pmc_bench.sh 'hash_write|hash_accum|hash_bwd_kernel' r3wrq "wrq sqw"
cat gpurun_out/pmc_r3wrq/wrq.txt
