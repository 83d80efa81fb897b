#!/bin/bash
# k_crc: issue-priority balancing on/off, with/without emission (B and C); stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 0 1048576 8 1048584 > $OUT/r04k_cmp_b.log 2>&1 || { tail -20 $OUT/r04k_cmp_b.log; exit 1; }
grep "k_crc<\|full pipeline" $OUT/r04k_cmp_b.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 1 cmp 0 1048576 8 1048584 > $OUT/r04k_cmp_c.log 2>&1 || { tail -20 $OUT/r04k_cmp_c.log; exit 1; }
grep "k_crc<\|full pipeline" $OUT/r04k_cmp_c.log
timeout -k 10 100 ./tools/kbench/kbench 1073741824 0 3 98 > $OUT/r04k_98.log 2>&1 || { tail -20 $OUT/r04k_98.log; exit 1; }
grep -A1 "emission stamps" $OUT/r04k_98.log | tail -2
for v in 520 1049096; do
timeout -k 10 100 ./tools/kbench/kbench 1073741824 0 3 $v > $OUT/r04k_$v.log 2>&1 || { tail -20 $OUT/r04k_$v.log; exit 1; }
grep -A12 "wave loop end" $OUT/r04k_$v.log | grep -v "^  xcd"
done
