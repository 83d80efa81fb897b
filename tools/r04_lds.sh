#!/bin/bash
# LDS pressure of k_crc variants: bank/address conflicts, LDS index-active cycles, FIFO-full, SALU cycles
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r04lds
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $*; do
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES -d "$OUT/v${v}" -o run --output-format csv -- \
      ./tools/kbench/kbench $((1 << 30)) ${MODE:-0} 3 $v > "$OUT/v${v}.log" 2>&1 || { tail -5 "$OUT/v${v}.log"; exit 1; }
done
