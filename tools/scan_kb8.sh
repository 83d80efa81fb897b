#!/bin/bash
# k_scan: 12- vs 8-wave builds (kbench scan mode), configs B and C, with phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${TAG:-kbs8}
mkdir -p "$OUT"
for b in ${BINS:-kbench kbench_w8}; do
for m in 0 1; do
  timeout -k 10 120 ./tools/kbench/$b 1073741824 $m scan ${VARS:-0 10 2058 512} > "$OUT/${b}_$m.log" 2>&1 || { tail -30 "$OUT/${b}_$m.log"; exit 1; }
  echo "== $b config $m"; grep "k_scan<" "$OUT/${b}_$m.log"; grep -A8 "entry" "$OUT/${b}_$m.log" | tail -9
done
done
