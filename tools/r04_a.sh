#!/bin/bash
# round 4: stream-verify k_crc bring-up: decode parity tests, then kbench (new vs round-3 window passes) on B and C.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_golden.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py > $OUT/r04a_tests.log 2>&1 || { tail -40 $OUT/r04a_tests.log; exit 1; }
tail -3 $OUT/r04a_tests.log
timeout -k 10 150 ./tools/kbench/kbench 1073741824 0 cmp 0 1048576 > $OUT/r04a_cmp_b.log 2>&1 || { tail -20 $OUT/r04a_cmp_b.log; exit 1; }
cat $OUT/r04a_cmp_b.log
timeout -k 10 150 ./tools/kbench/kbench 1073741824 1 cmp 0 1048576 > $OUT/r04a_cmp_c.log 2>&1 || { tail -20 $OUT/r04a_cmp_c.log; exit 1; }
cat $OUT/r04a_cmp_c.log
