#!/bin/bash
# k_crc ablations on config B: times + instruction counts + wave states
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 0 8388608 10485760 2097152 8 > $OUT/r04g_cmp_b.log 2>&1 || { tail -20 $OUT/r04g_cmp_b.log; exit 1; }
grep "k_crc<\|full pipeline\|k_chase  " $OUT/r04g_cmp_b.log
timeout -k 10 100 ./tools/kbench/kbench 1073741824 0 spat > $OUT/r04g_spat.log 2>&1 || { tail -20 $OUT/r04g_spat.log; exit 1; }
tail -3 $OUT/r04g_spat.log
bash tools/r04_pmc2.sh 0 8388608 10485760 > /dev/null && bash tools/r04_pmc3.sh 0 8388608 10485760 > /dev/null
