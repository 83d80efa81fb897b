#!/bin/bash
# PMC counter passes over the product k_crc (kbench counter mode), one counter set per pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/pmc_kcrc
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
while read -r set; do
  [[ -z $set ]] && continue
  i=$((i + 1))
  timeout -k 10 240 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- \
    ./tools/kbench/kbench $((1 << 30)) ${MODE:-0} 5 > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
done <<SETS
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
FETCH_SIZE
WRITE_SIZE
SETS
find "$OUT" -name "*counter_collection*"
