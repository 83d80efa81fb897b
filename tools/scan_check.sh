#!/bin/bash
# k_scan bring-up session: decode parity (both paths), full-size parity at configs A/B/C, a short bench.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${TAG:-s1}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 120 --timeout-method thread \
  > "$OUT/t1.log" 2>&1 || { echo "t1 failed"; tail -30 "$OUT/t1.log"; exit 1; }
tail -2 "$OUT/t1.log"
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread \
  -k "${FULLK:-config_b or config_c or config_a}" > "$OUT/t2.log" 2>&1 || { echo "t2 failed"; tail -30 "$OUT/t2.log"; exit 1; }
tail -2 "$OUT/t2.log"
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --decode-path 0 ${BENCH_ARGS:-} > "$OUT/b1.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/b1.log"; exit 1; }
tail -1 "$OUT/b1.log" | cut -c1-1200
