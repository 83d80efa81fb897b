#!/bin/bash
# VALU / SALU / LDS instruction counts of k_crc variants (one pass each)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r04pmc2
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $*; do
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH -d "$OUT/v${v}" -o run --output-format csv -- \
      ./tools/kbench/kbench $((1 << 30)) ${MODE:-0} 1 $v > "$OUT/v${v}.log" 2>&1 || { tail -5 "$OUT/v${v}.log"; exit 1; }
done
