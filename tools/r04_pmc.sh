#!/bin/bash
# SQ counters of k_crc variants (kbench counter mode), one counter set per rocprofv3 pass
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r04pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $*; do
  i=0
  while read -r set; do
    [[ -z $set ]] && continue
    i=$((i + 1))
    timeout -k 10 120 rocprofv3 --pmc $set -d "$OUT/v${v}_p$i" -o run --output-format csv -- \
      ./tools/kbench/kbench $((1 << 30)) 0 1 $v > "$OUT/v${v}_p$i.log" 2>&1 || { tail -20 "$OUT/v${v}_p$i.log"; exit 1; }
  done <<SETS
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SETS
  timeout -k 10 120 rocprofv3 --pmc SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU -d "$OUT/v${v}_p3" -o run --output-format csv -- \
      ./tools/kbench/kbench $((1 << 30)) 0 1 $v > "$OUT/v${v}_p3.log" 2>&1 || tail -5 "$OUT/v${v}_p3.log"
done
find "$OUT" -name "*counter_collection*" | head -3
