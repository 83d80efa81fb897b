#!/bin/bash
# k_scan timing probes (kbench scan mode) on the 12-wave build, then variant 10 on the 16-wave build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${TAG:-kbs4}
mkdir -p "$OUT"
for m in 0 1; do
  timeout -k 10 120 ./tools/kbench/kbench 1073741824 $m scan ${VARS:-0 10 11 42 512} > "$OUT/kb_$m.log" 2>&1 || { tail -30 "$OUT/kb_$m.log"; exit 1; }
  echo "== config $m"; grep "k_scan<" "$OUT/kb_$m.log"; grep -A8 "entry" "$OUT/kb_$m.log" | tail -9
done
timeout -k 10 120 ./tools/kbench/kbench_w16 1073741824 0 scan 10 11 42 > "$OUT/kb16.log" 2>&1 || { tail -30 "$OUT/kb16.log"; exit 1; }
echo "== w16"; grep "k_scan<" "$OUT/kb16.log"
