#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r04tq; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/kbench/kbench 1073741824 0 seq 60 -1 > $OUT/seq_noev.log 2>&1 && tail -1 $OUT/seq_noev.log
rm -rf $OUT/kb
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/kb -o run --output-format csv -- ./tools/kbench/kbench 1073741824 0 seq 60 -1 > $OUT/kb.log 2>&1 || { tail -20 $OUT/kb.log; exit 1; }
