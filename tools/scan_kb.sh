#!/bin/bash
# k_scan timing probes (kbench scan mode), config B and C, variants in VARS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${TAG:-kbs}
mkdir -p "$OUT"
for m in 0 1; do
  timeout -k 10 120 ./tools/kbench/kbench 1073741824 $m scan ${VARS:-0 2058 512} > "$OUT/kb_$m.log" 2>&1 || { tail -30 "$OUT/kb_$m.log"; exit 1; }
  echo "== config $m"; grep "k_scan<" "$OUT/kb_$m.log"; grep -A8 "entry" "$OUT/kb_$m.log" | tail -9
done
