#!/bin/bash
# k_crc: emission-first waves 0/1/2/4/6 (B and C), stamps of the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 268435456 536870912 805306368 1342177280 1879048192 8 > $OUT/r04j_cmp_b.log 2>&1 || { tail -20 $OUT/r04j_cmp_b.log; exit 1; }
grep "k_crc<\|full pipeline" $OUT/r04j_cmp_b.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 1 cmp 268435456 805306368 1342177280 8 > $OUT/r04j_cmp_c.log 2>&1 || { tail -20 $OUT/r04j_cmp_c.log; exit 1; }
grep "k_crc<\|full pipeline" $OUT/r04j_cmp_c.log
timeout -k 10 100 ./tools/kbench/kbench 1073741824 0 3 98 > $OUT/r04j_98.log 2>&1 || { tail -20 $OUT/r04j_98.log; exit 1; }
grep -A1 "emission stamps" $OUT/r04j_98.log | tail -2
