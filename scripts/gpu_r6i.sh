# Round 6: the summary kernel's tests, then capture order of the step's forks (NGP_MAIN_FIRST bits: 1 round 2
# before the march branch, 2 MLP backward before the bucket plan, 4 accumulation before the coarse branch),
# alternating 1000-step windows, and one wave timeline of the best guess.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6i; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "summary or march or trainer" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/ab_env.sh r6i 3 "||" "|NGP_MAIN_FIRST=1|" "|NGP_MAIN_FIRST=7|" "|NGP_MAIN_FIRST=6|"
NGP_MAIN_FIRST=7 timeout -k 10 300 python -u scripts/diag/wave_timeline.py 2 > $OUT/wave_timeline_mf7.txt 2> $OUT/wave_timeline.err || true
head -22 $OUT/wave_timeline_mf7.txt | cut -c1-160
