#!/bin/bash
# kbench session: config B diagnostics, k_crc variant compare (B), config C compare. Each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 240 ./tools/kbench/kbench > $OUT/kb_b.log 2>&1 || { tail -20 $OUT/kb_b.log; exit 1; }
timeout -k 10 120 ./tools/kbench/kbench 1073741824 0 cmp ${VARS:-0 8 2048} > $OUT/kb_cmp_b.log 2>&1 || { tail -20 $OUT/kb_cmp_b.log; exit 1; }
timeout -k 10 120 ./tools/kbench/kbench 1073741824 1 cmp ${VARS:-0 8 2048} > $OUT/kb_cmp_c.log 2>&1 || { tail -20 $OUT/kb_cmp_c.log; exit 1; }
echo kb done
