# Round 6: test-time render, this tree vs the round-5 tree (abtree_r5, built in place): the same 2000-step
# training then 20 frames at 800x800, alternating; then a kernel trace of each for per-kernel times.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${1:-r6m}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for tree in . abtree_r5; do
    n=$(basename $(cd $tree && pwd))
    (cd $tree && timeout -k 10 200 python -u scripts/render_profile.py --pretrain 2000 --frames 20 > $OUT/render_${n}_$rep.txt 2> $OUT/render_${n}_$rep.err)
    echo "$tree rep$rep $(tail -1 $OUT/render_${n}_$rep.txt | cut -c1-300)"
  done
done
for tree in . abtree_r5; do
  n=$(basename $(cd $tree && pwd))
  (cd $tree && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_$n -o run -f csv -- python3 scripts/render_profile.py --pretrain 2000 --frames 10 > $OUT/prof_render_$n.txt 2> $OUT/prof_render_$n.err)
  TR=$(find $OUT/prof_$n -name 'run_kernel_trace.csv' | head -1)
  python3 scripts/render_kstats.py $TR 10 > $OUT/render_kstats_$n.txt 2>&1 || true
  rm -rf $OUT/prof_$n
  echo "== $tree"; head -14 $OUT/render_kstats_$n.txt | cut -c1-150
done
