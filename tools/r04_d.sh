#!/bin/bash
# round 4: stream-verify parity (decode tests), kbench B/C, SQ counters of the product k_crc
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_golden.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py > $OUT/r04d_tests.log 2>&1 || { tail -40 $OUT/r04d_tests.log; exit 1; }
tail -2 $OUT/r04d_tests.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 0 1048576 4194304 8388608 10485760 67108864 > $OUT/r04d_cmp_b.log 2>&1 || { tail -20 $OUT/r04d_cmp_b.log; exit 1; }
grep "k_crc<\|full pipeline\|k_chase  " $OUT/r04d_cmp_b.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 1 cmp 0 1048576 > $OUT/r04d_cmp_c.log 2>&1 || { tail -20 $OUT/r04d_cmp_c.log; exit 1; }
grep "k_crc<\|full pipeline\|k_chase  " $OUT/r04d_cmp_c.log
bash tools/r04_pmc.sh 0 > /dev/null
