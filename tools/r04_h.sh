#!/bin/bash
# k_crc: emission / chain / slow-path ablations and per-wave end stamps on config B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 0 8 8388616 10485760 10485768 > $OUT/r04h_cmp_b.log 2>&1 || { tail -20 $OUT/r04h_cmp_b.log; exit 1; }
grep "k_crc<" $OUT/r04h_cmp_b.log
timeout -k 10 100 ./tools/kbench/kbench 1073741824 0 3 520 > $OUT/r04h_520.log 2>&1 || { tail -20 $OUT/r04h_520.log; exit 1; }
grep -A12 "wave loop end" $OUT/r04h_520.log
timeout -k 10 100 ./tools/kbench/kbench 1073741824 0 3 10486280 > $OUT/r04h_fast.log 2>&1 || { tail -20 $OUT/r04h_fast.log; exit 1; }
grep -A12 "wave loop end" $OUT/r04h_fast.log
