#!/bin/bash
# A/B of encode builds on config E: `bash tools/ab_events.sh a b ...` runs tools/bench_encode.py once per
# bitcaskdb_amd/libbcw_<name>.so (loaded through BCW_LIB) and prints per-kernel times. Build the variants
# in this container first (copy libbcw.so after each `python bitcaskdb_amd/build.py`).
set -o pipefail
for v in "$@"; do
  BCW_LIB=$PWD/bitcaskdb_amd/libbcw_$v.so timeout -k 10 300 python -u tools/bench_encode.py --records 10000000 --steps 2 \
    > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  echo "$v $(grep -o '"kernel_ms": {[^}]*}' gpurun_out/ab_$v.log) $(grep -o '"encode_ms": [0-9.]*' gpurun_out/ab_$v.log)"
done
