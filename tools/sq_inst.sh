#!/bin/bash
# Dynamic instruction mix of k_crc (tools/kbench counter mode, 5 launches of the product k_crc at config B):
# SQ_INSTS_* per pass, GRBM_GUI_ACTIVE for the effective clock.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES"; do
  i=$((i+1))
  rm -rf $OUT/si$i
  timeout -s KILL 60 rocprofv3 --pmc $set -d $OUT/si$i -o run --output-format csv -- ./tools/kbench/kbench 1073741824 0 5 \
    > $OUT/si$i.log 2>&1 || { tail -20 $OUT/si$i.log; exit 1; }
done
echo done
