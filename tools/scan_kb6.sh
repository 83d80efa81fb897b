#!/bin/bash
# k_scan window-phase overheads: lane operator + scan (1024), prefix stores (2048), concurrent chase (4096).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${TAG:-kbs6}
mkdir -p "$OUT"
for m in 0 1; do
  timeout -k 10 120 ./tools/kbench/kbench 1073741824 $m scan 10 1034 2058 4106 7178 7179 11 > "$OUT/kb_$m.log" 2>&1 || { tail -30 "$OUT/kb_$m.log"; exit 1; }
  echo "== config $m"; grep "k_scan<" "$OUT/kb_$m.log"
done
timeout -k 10 200 ./tools/kbench/kbench > "$OUT/kb_diag.log" 2>&1 || { tail -30 "$OUT/kb_diag.log"; exit 1; }
grep -E "stream read|loads only|depth:|d1 by|core" "$OUT/kb_diag.log"
