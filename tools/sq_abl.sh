#!/bin/bash
# VALU / LDS / SALU instruction counts of k_crc ablation variants (tools/kbench counter mode, config B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for v in ${VARIANTS:-0 1 2 4 8 128 256 384}; do
  timeout -k 10 60 ./tools/kbench/kbench 1073741824 0 3 $v 2>&1 | grep done || exit 1
  rm -rf $OUT/sa$v
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    -d $OUT/sa$v -o run --output-format csv -- ./tools/kbench/kbench 1073741824 0 3 $v > $OUT/sa$v.log 2>&1 || { tail -20 $OUT/sa$v.log; exit 1; }
  grep "done" $OUT/sa$v.log
done
echo done
