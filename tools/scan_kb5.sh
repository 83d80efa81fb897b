#!/bin/bash
# k_scan: window-phase time by the number of streaming waves (kbench scan mode, variants 10/138/266 and no-chain).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${TAG:-kbs5}
mkdir -p "$OUT"
for b in kbench kbench_w16; do
for m in 0 1; do
  timeout -k 10 120 ./tools/kbench/$b 1073741824 $m scan 10 138 266 11 139 267 > "$OUT/${b}_$m.log" 2>&1 || { tail -30 "$OUT/${b}_$m.log"; exit 1; }
  echo "== $b config $m"; grep "k_scan<" "$OUT/${b}_$m.log"
done
done
