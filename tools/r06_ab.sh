# A/B of two kbench builds on one box (tools/kbench/kbench_head = the last commit, kbench = the tree), then the
# per-XCD split on / off in pipelines (kbench xbal). Output under gpurun_out/$TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT; TAG=${TAG:-r06ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
for b in kbench_head kbench; do
  echo "== $b rep $rep"
  KB_CLOCK=1 timeout -k 10 200 tools/kbench/$b $((1<<30)) 0 cmp 0 8 > $OUT/${b}_$rep.log 2>&1 || exit 1
  grep -E "full pipeline|^  k_c|timeline: pipeline|k_crc<" $OUT/${b}_$rep.log | head -12
done
done
for m in 0 1; do
  echo "== xbal config $m"
  timeout -k 10 300 tools/kbench/kbench $((1 << 30)) $m xbal > $OUT/xbal_$m.log 2>&1 || exit 1
  grep xbal $OUT/xbal_$m.log
done
