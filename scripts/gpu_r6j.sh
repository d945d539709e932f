# Round 6: hardware queues per process (HIP's default 4: the step graph's parallel branches and the
# trainer's streams share them round-robin) x capture order of the step's forks; alternating 1000-step windows.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6j; mkdir -p $OUT
bash scripts/ab_env.sh r6j 3 "||" "|GPU_MAX_HW_QUEUES=8|" "|GPU_MAX_HW_QUEUES=8 NGP_MAIN_FIRST=7|" "|GPU_MAX_HW_QUEUES=16|" "|GPU_MAX_HW_QUEUES=8 NGP_MAIN_FIRST=1|"
GPU_MAX_HW_QUEUES=8 NGP_MAIN_FIRST=7 timeout -k 10 300 python -u scripts/diag/wave_timeline.py 2 > $OUT/wave_timeline_q8_mf7.txt 2> $OUT/wave_timeline.err || true
sed -n 20,45p $OUT/wave_timeline_q8_mf7.txt | cut -c1-160
