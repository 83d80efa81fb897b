#!/bin/bash
# Diagnostics session: kbench config B and C (phase stamps, k_chase ablations), the header-hop latency probe,
# and the shipped k_crc's SQ / TA / TCP / TCC counters (kbench counter mode: 5 launches of the product k_crc),
# one rocprofv3 --pmc pass per counter set. Every GPU step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/diag
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-kb,chase,pmc}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has kb; then
  timeout -k 10 240 ./tools/kbench/kbench > "$OUT/kb_b.log" 2>&1 || { tail -20 "$OUT/kb_b.log"; exit 1; }
  timeout -k 10 240 ./tools/kbench/kbench 1073741824 1 > "$OUT/kb_c.log" 2>&1 || { tail -20 "$OUT/kb_c.log"; exit 1; }
fi
if has chase; then
  timeout -k 10 60 ./tools/kbench/chasebench > "$OUT/chase.log" 2>&1 || { tail -20 "$OUT/chase.log"; exit 1; }
fi
if has pmc; then
  i=0
  while read -r set; do
    [[ -z $set ]] && continue
    i=$((i + 1))
    rm -rf "$OUT/p$i"
    timeout -s KILL 90 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- \
      ./tools/kbench/kbench 1073741824 0 5 > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
  done <<SETS
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
TCC_REQ_sum TCC_HIT_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
FETCH_SIZE
WRITE_SIZE
SETS
fi
echo "diag done"
