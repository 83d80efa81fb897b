#!/bin/bash
# k_crc (balanced stream): emission costs; emission-only variants (parse / prefix loads)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 0 8 4096 8192 32768 36864 40960 > $OUT/r04m_cmp_b.log 2>&1 || { tail -20 $OUT/r04m_cmp_b.log; exit 1; }
grep "k_crc<\|full pipeline" $OUT/r04m_cmp_b.log
