#!/bin/bash
# k_crc with per-XCD emission queues: decode parity subset, kbench B/C, stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_golden.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_host.py > $OUT/r04n_tests.log 2>&1 || { tail -40 $OUT/r04n_tests.log; exit 1; }
tail -1 $OUT/r04n_tests.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp 0 8 32768 > $OUT/r04n_cmp_b.log 2>&1 || { tail -20 $OUT/r04n_cmp_b.log; exit 1; }
grep "k_crc<\|full pipeline" $OUT/r04n_cmp_b.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 1 cmp 0 8 > $OUT/r04n_cmp_c.log 2>&1 || { tail -20 $OUT/r04n_cmp_c.log; exit 1; }
grep "k_crc<\|full pipeline" $OUT/r04n_cmp_c.log
timeout -k 10 100 ./tools/kbench/kbench 1073741824 0 3 98 > $OUT/r04n_98.log 2>&1 || { tail -20 $OUT/r04n_98.log; exit 1; }
grep -A1 "emission stamps" $OUT/r04n_98.log | tail -2
