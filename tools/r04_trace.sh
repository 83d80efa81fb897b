#!/bin/bash
# per-dispatch durations: bench.py (60 timed steps) under kernel-trace, and kbench seq, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r04t; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/kbench/kbench 1073741824 0 seq 40 > $OUT/seq.log 2>&1 || { tail -5 $OUT/seq.log; exit 1; }
tail -1 $OUT/seq.log
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- \
  python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-extras --inflight 1 --event-every 1000 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
