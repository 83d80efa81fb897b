#!/bin/bash
# round 4: decode parity subset, kbench B/C, instruction counts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_golden.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_host.py > $OUT/r04f_tests.log 2>&1 || { tail -40 $OUT/r04f_tests.log; exit 1; }
tail -2 $OUT/r04f_tests.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 0 4194304 8388608 8 > $OUT/r04f_cmp_b.log 2>&1 || { tail -20 $OUT/r04f_cmp_b.log; exit 1; }
grep "k_crc<\|full pipeline\|k_chase  " $OUT/r04f_cmp_b.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 1 cmp 0 8 > $OUT/r04f_cmp_c.log 2>&1 || { tail -20 $OUT/r04f_cmp_c.log; exit 1; }
grep "k_crc<\|full pipeline\|k_chase  " $OUT/r04f_cmp_c.log
bash tools/r04_pmc2.sh 0 > /dev/null
