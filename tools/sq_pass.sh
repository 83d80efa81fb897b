#!/bin/bash
# SQ counters of k_crc alone (tools/kbench counter mode: 5 launches of the product k_crc after setup),
# in separate rocprofv3 --pmc passes (8 SQ counters at most per pass), then config C on bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  rm -rf $OUT/sq$i
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/sq$i -o run --output-format csv -- ./tools/kbench/kbench 1073741824 0 5 \
    > $OUT/sq$i.log 2>&1 || { tail -20 $OUT/sq$i.log; exit 1; }
done
timeout -k 10 300 python3 bench.py --config C --no-extras > $OUT/bench_c.log 2>&1 || { tail -20 $OUT/bench_c.log; exit 1; }
tail -1 $OUT/bench_c.log | cut -c1-300
echo done
