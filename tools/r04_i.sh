#!/bin/bash
# k_crc: emission timing (stamps), emission alone, no-emission wave ends
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 0 32768 8 > $OUT/r04i_cmp_b.log 2>&1 || { tail -20 $OUT/r04i_cmp_b.log; exit 1; }
grep "k_crc<" $OUT/r04i_cmp_b.log
for v in 98 97 520; do
timeout -k 10 100 ./tools/kbench/kbench 1073741824 0 3 $v > $OUT/r04i_$v.log 2>&1 || { tail -20 $OUT/r04i_$v.log; exit 1; }
grep -A12 "wave loop end\|emission stamps" $OUT/r04i_$v.log | grep -v "^  xcd"
done
