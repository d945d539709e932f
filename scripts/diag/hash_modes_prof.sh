# Kernel durations (rocprofv3 stats) of the coarse atomic hash backward
# levels 0-8 under diagnostic modes 0 / 1 / 3 (stages.py workloads).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for m in 0 1; do
  NGP_HASH_BWD_MODE=$m PRETRAIN=1000 NGP_STAGES_ONLY=coarse timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/hm$m -o run -f csv -- python3 scripts/diag/stages.py > /dev/null 2>&1
  echo "mode $m"
  grep -i "hash_bwd_kernel" gpurun_out/hm$m/run_kernel_stats.csv | cut -c1-200
  rm -f gpurun_out/hm$m/run_kernel_trace.csv
done
