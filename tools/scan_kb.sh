#!/bin/bash
# k_scan phase breakdown (tools/kbench scan mode): ablation variants interleaved, per-wave phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${TAG:-kbs}
mkdir -p "$OUT"
timeout -k 10 120 ./tools/kbench/kbench 1073741824 0 scan ${VARS:-0 1 2 4 8 10 14 512} > "$OUT/b.log" 2>&1 || { tail -30 "$OUT/b.log"; exit 1; }
tail -40 "$OUT/b.log"
timeout -k 10 120 ./tools/kbench/kbench 1073741824 1 scan ${VARS:-0 1 2 4 8 10 14 512} > "$OUT/c.log" 2>&1 || { tail -30 "$OUT/c.log"; exit 1; }
tail -40 "$OUT/c.log"
