# Round 6 (third session): the test render's loop decision made by the compositing launch's last workgroup
# (ngp_render_test_composite_decide / _march_decided: one launch fewer per iteration).  Renderer tests first
# (bit-exact vs the host loop), then the render harness on the tree and on HEAD's library + renderer.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6aq; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_renderer_gpu.py tests/test_golden_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_render.log 2>&1
tail -1 $OUT/pytest_render.log
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/diag/render_graph_sizes.py --reps 2 --configs 24:4 > $OUT/tree_$rep.txt 2> $OUT/tree_$rep.err
  (cd abtree_base && NGP_AMD_LIB=$GRAFT_REPO_ROOT/abtree_base/ar-nerf_amd/lib/libngp_amd.so timeout -k 10 300 python -u scripts/diag/render_graph_sizes.py --reps 2 --configs 24:4 > $GRAFT_REPO_ROOT/$OUT/base_$rep.txt 2> $GRAFT_REPO_ROOT/$OUT/base_$rep.err)
done
grep -h "rep" $OUT/tree_*.txt $OUT/base_*.txt
