#!/bin/bash
# One GPU session for the encode path: parity tests, then the config-E bench (10 M records). Every GPU
# step has its own time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out
mkdir -p "$OUT"
RECORDS=${RECORDS:-10000000}
echo "== encode tests ($(date +%T))"
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 120 --timeout-method thread \
  > "$OUT/enc_tests.log" 2>&1 || { tail -30 "$OUT/enc_tests.log"; exit 1; }
tail -2 "$OUT/enc_tests.log"
echo "== encode bench ($(date +%T))"
timeout -k 10 400 python -u tools/bench_encode.py --records "$RECORDS" --out "$OUT/r01_encode_bench.json" \
  > "$OUT/benc.log" 2>&1 || { tail -30 "$OUT/benc.log"; exit 1; }
tail -1 "$OUT/benc.log"
echo "== done ($(date +%T))"
