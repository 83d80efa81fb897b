#!/bin/bash
# A/B of two kbench builds (kbench_old vs kbench), alternating processes; config B and C; k_crc full and no emission
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r04ab; mkdir -p $OUT
for r in 1 2 3; do
  for b in kbench_old kbench; do
    for m in 0 1; do
      timeout -k 10 120 ./tools/kbench/$b 1073741824 $m cmp 0 8 > $OUT/${b}_m${m}_r$r.log 2>&1 || { tail -5 $OUT/${b}_m${m}_r$r.log; exit 1; }
      echo "$b mode $m round $r: $(grep 'k_crc<' $OUT/${b}_m${m}_r$r.log | awk '{print $1, $5}' | tr '\n' ' ')"
    done
  done
done
