#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r04tp; mkdir -p $OUT
export TMPDIR=/tmp
for a in torch hip; do
  rm -rf $OUT/$a
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/$a -o run --output-format csv -- python3 tools/trace_probe.py $a 30 > $OUT/$a.log 2>&1 || { tail -20 $OUT/$a.log; exit 1; }
done
