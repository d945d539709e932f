# Round 5: the data-parallel step's cost on one GPU (VERDICT r04 Next #5): the world-8 step emulated
# (--emulate-dp 8: ZeRO-1 buckets, the collectives as local copies, whole step captured as one graph) at
# K = 1, 2, 4 fine buckets against the single-process step, alternating; then a rocprofv3 timeline of the
# K = 2 emulated step.
# usage: gpurun -- bash scripts/gpu_r5v.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5v}
mkdir -p gpurun_out/$T
bash scripts/ab_env.sh $T/ab 2 "||--steps 600" "||--steps 600 --emulate-dp 8 --dp-fine-buckets 2" \
    "||--steps 600 --emulate-dp 8 --dp-fine-buckets 4" "||--steps 600 --emulate-dp 8 --dp-fine-buckets 1"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T/prof -o run -f csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 --infer-frames 0 --no-oracle-quality --dropin-steps 0 --breakdown-steps 20 --emulate-dp 8 --dp-fine-buckets 2 > gpurun_out/$T/prof_bench.json 2> gpurun_out/$T/prof_bench.err
python3 scripts/timeline.py $(find gpurun_out/$T/prof -name 'run_kernel_trace.csv' | head -1) 20 10 sample_batch_kernel > gpurun_out/$T/timeline_emulate_dp8_k2.txt 2>&1 || true
rm -rf gpurun_out/$T/prof
head -30 gpurun_out/$T/timeline_emulate_dp8_k2.txt
