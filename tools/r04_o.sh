#!/bin/bash
# k_crc slow-path ablations (no emission): close / split op / masks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 0 8 65544 131080 262152 458760 8388616 > $OUT/r04o_cmp_b.log 2>&1 || { tail -20 $OUT/r04o_cmp_b.log; exit 1; }
grep "k_crc<\|full pipeline" $OUT/r04o_cmp_b.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 1 cmp 0 8 65544 131080 262152 458760 8388616 > $OUT/r04o_cmp_c.log 2>&1 || { tail -20 $OUT/r04o_cmp_c.log; exit 1; }
grep "k_crc<\|full pipeline" $OUT/r04o_cmp_c.log
