#!/bin/bash
# round 4: stream-verify parity (decode tests) + ablations
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_golden.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py > $OUT/r04c_tests.log 2>&1 || { tail -40 $OUT/r04c_tests.log; exit 1; }
tail -2 $OUT/r04c_tests.log
V="${VARS:-0 1048576 2097152 4194304 8388608 10485760 8 33554432 100663296}"
timeout -k 10 200 ./tools/kbench/kbench 1073741824 0 cmp $V > $OUT/r04c_cmp_b.log 2>&1 || { tail -20 $OUT/r04c_cmp_b.log; exit 1; }
grep "k_crc<\|full pipeline\|k_chase  " $OUT/r04c_cmp_b.log
timeout -k 10 200 ./tools/kbench/kbench 1073741824 1 cmp 0 1048576 > $OUT/r04c_cmp_c.log 2>&1 || { tail -20 $OUT/r04c_cmp_c.log; exit 1; }
grep "k_crc<\|full pipeline\|k_chase  " $OUT/r04c_cmp_c.log
