#!/bin/bash
# A/B of two kbench builds (tools/kbench/kbench_old: the previous commit's sources; kbench: the working tree),
# alternating processes, configs B (mode 0) and C (mode 1): pipeline, k_crc alone and k_chase variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r04ab; mkdir -p $OUT
for r in 1 2; do
  for b in kbench_old kbench; do
    for m in 0 1; do
      timeout -k 10 150 ./tools/kbench/$b 1073741824 $m > $OUT/${b}_m${m}_r$r.log 2>&1 || { tail -5 $OUT/${b}_m${m}_r$r.log; exit 1; }
      echo "$b mode $m round $r: $(grep -h 'full pipeline\|^k_chase alone' $OUT/${b}_m${m}_r$r.log | tr '\n' ' ')"
    done
  done
done
