#!/bin/bash
# Memory-pipeline counters (TA / TCP / TCC) of k_crc variants (tools/kbench counter mode, config B), one
# rocprofv3 --pmc pass per counter group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for v in ${VARIANTS:-0 32}; do
  i=0
  for set in "TCC_REQ_sum TCC_HIT_sum TCC_READ_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
             "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
             "TCP_TCC_READ_REQ_LATENCY_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TOTAL_READ_sum TD_TD_BUSY_sum TA_BUSY_avr"; do
    i=$((i+1))
    rm -rf $OUT/mp${v}_$i
    timeout -s KILL 60 rocprofv3 --pmc $set -d $OUT/mp${v}_$i -o run --output-format csv -- ./tools/kbench/kbench 1073741824 0 3 $v \
      > $OUT/mp${v}_$i.log 2>&1 || { tail -20 $OUT/mp${v}_$i.log; exit 1; }
  done
  grep done $OUT/mp${v}_1.log
done
echo done
