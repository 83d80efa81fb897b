#!/bin/bash
# round 4: stream-verify ablations (kbench cmp, config B then C)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
V="${VARS:-0 1048576 2097152 4194304 8388608 10485760 8 8388616 33554432 100663296 134217728}"
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp $V > $OUT/r04b_cmp_b.log 2>&1 || { tail -20 $OUT/r04b_cmp_b.log; exit 1; }
grep "k_crc<" $OUT/r04b_cmp_b.log
