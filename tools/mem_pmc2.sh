#!/bin/bash
# TCP -> TCC request counts and TA busy of the product k_crc in several kbench builds (config B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for b in ${BINS:-kbench_ref kbench}; do
  rm -rf $OUT/m2_$b
  timeout -s KILL 60 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE \
    -d $OUT/m2_$b -o run --output-format csv -- ./tools/kbench/$b 1073741824 0 3 0 > $OUT/m2_$b.log 2>&1 || { tail -20 $OUT/m2_$b.log; exit 1; }
done
echo done
