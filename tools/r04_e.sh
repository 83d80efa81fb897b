#!/bin/bash
# round 4: full GPU suite, then kbench B/C and the product k_crc's SQ counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $OUT/r04e_tests.log 2>&1 || { tail -60 $OUT/r04e_tests.log; exit 1; }
tail -3 $OUT/r04e_tests.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 0 4194304 8388608 10485760 8 67108864 > $OUT/r04e_cmp_b.log 2>&1 || { tail -20 $OUT/r04e_cmp_b.log; exit 1; }
grep "k_crc<\|full pipeline\|k_chase  " $OUT/r04e_cmp_b.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 1 cmp 0 8 > $OUT/r04e_cmp_c.log 2>&1 || { tail -20 $OUT/r04e_cmp_c.log; exit 1; }
grep "k_crc<\|full pipeline\|k_chase  " $OUT/r04e_cmp_c.log
bash tools/r04_pmc.sh 0 > /dev/null
