#!/bin/bash
# Round 5 iteration run: GPU parity tests (TESTS, default the whole -m gpu suite), then kbench k_crc variants with the
# in-kernel clock for config B and C (VARIANTS, default "0 8 8388616"). Output under gpurun_out/r05it/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05it
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
VARIANTS=${VARIANTS:-0 8 8388616}
if [[ "$TESTS" != "none" ]]; then
  echo "== tests $(date +%T)"
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -2 "$OUT/gpu_tests.log"
fi
for m in 0 1; do
  echo "== kbench cmp config $m $(date +%T)"
  KB_CLOCK=1 timeout -k 10 300 tools/kbench/kbench $((1 << 30)) $m cmp $VARIANTS > "$OUT/cmp_$m.log" 2>&1 || { tail -5 "$OUT/cmp_$m.log"; exit 1; }
  grep -E "k_crc<|recheck" "$OUT/cmp_$m.log"
done
echo "== seqk from idle $(date +%T)"
KB_CLOCK=1 KB_IDLE_MS=1000 timeout -k 10 120 tools/kbench/kbench $((1 << 30)) 0 seqk 60 0 > "$OUT/seqk.log" 2>&1 || { tail -5 "$OUT/seqk.log"; exit 1; }
grep seqk "$OUT/seqk.log" | cut -c1-400
