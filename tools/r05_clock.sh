#!/bin/bash
# Round 5: in-kernel clock (shader cycles / real time per k_crc launch) across 80 back-to-back launches started from an
# idle chip (KB_IDLE_MS) and from a busy one.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05c
rm -rf "$OUT"; mkdir -p "$OUT"
KB=tools/kbench/kbench
for idle in 1000 0; do
  for v in 0 8; do
    echo "== seqk $v idle $idle $(date +%T)"
    KB_CLOCK=1 KB_IDLE_MS=$idle timeout -k 10 120 $KB $((1 << 30)) 0 seqk 80 $v > "$OUT/seqk_${v}_idle${idle}.log" 2>&1 || { tail -5 "$OUT/seqk_${v}_idle${idle}.log"; exit 1; }
    grep -E "seqk" "$OUT/seqk_${v}_idle${idle}.log"
  done
done
echo "== config C $(date +%T)"
KB_CLOCK=1 KB_IDLE_MS=1000 timeout -k 10 120 $KB $((1 << 30)) 1 seqk 80 0 > "$OUT/seqk_c.log" 2>&1 || { tail -5 "$OUT/seqk_c.log"; exit 1; }
grep -E "seqk" "$OUT/seqk_c.log"
