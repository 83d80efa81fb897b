#!/bin/bash
# k_scan iteration: decode parity (both paths) + full-size A/B/C, then the kbench phase breakdown (B, C).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${TAG:-it}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 60 --timeout-method thread \
  > "$OUT/t1.log" 2>&1 || { echo "t1 failed"; tail -30 "$OUT/t1.log"; exit 1; }
tail -1 "$OUT/t1.log"
BCW_TEST_DECODE_PATH=${DP:-0} timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread \
  -k "${FULLK:-config_b or config_c or config_a}" > "$OUT/t2.log" 2>&1 || { echo "t2 failed"; tail -30 "$OUT/t2.log"; exit 1; }
tail -1 "$OUT/t2.log"
for m in 0 1; do
  timeout -k 10 120 ./tools/kbench/kbench 1073741824 $m scan ${VARS:-0 2 8 10 512} > "$OUT/kb_$m.log" 2>&1 || { tail -30 "$OUT/kb_$m.log"; exit 1; }
  echo "== config $m"; grep "k_scan<" "$OUT/kb_$m.log"; grep -A8 "entry" "$OUT/kb_$m.log" | tail -9
done
