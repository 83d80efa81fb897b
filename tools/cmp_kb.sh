#!/bin/bash
# A/B of kbench builds (tools/kbench/kbench_*): k_crc timing per variant + SQ / instruction-cache counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for b in ${BINS:-kbench_ref kbench kbench_ab}; do
  for v in 0 2 1; do timeout -k 10 60 ./tools/kbench/$b 1073741824 0 3 $v 2>&1 | grep done | sed "s/^/$b /" || exit 1; done
  rm -rf $OUT/ck_$b
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS \
    -d $OUT/ck_$b -o run --output-format csv -- ./tools/kbench/$b 1073741824 0 3 0 > $OUT/ck_$b.log 2>&1 || { tail -20 $OUT/ck_$b.log; exit 1; }
done
echo done
