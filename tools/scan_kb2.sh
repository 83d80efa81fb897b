#!/bin/bash
# k_scan window-phase probes: 12- and 16-wave builds, dynamic vs static units, with/without P stores.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${TAG:-kbs2}
mkdir -p "$OUT"
for b in kbench kbench_w16; do
  for m in 0 1; do
    timeout -k 10 120 ./tools/kbench/$b 1073741824 $m scan ${VARS:-10 42 74 106 11 43 14} > "$OUT/${b}_$m.log" 2>&1 || { tail -30 "$OUT/${b}_$m.log"; exit 1; }
    echo "== $b config $m"; grep "k_scan<" "$OUT/${b}_$m.log"
  done
done
