#!/bin/bash
# k_pack phase ablations on config E (BCW_PACK_ABL bits: 1 no CRC, 2 no copy, 8 no store). Ablated runs
# fail the parity check by design (exit 1); any other failure stops the chain.
set -o pipefail
for a in "$@"; do
  BCW_PACK_ABL=$a timeout -k 10 300 python -u tools/bench_encode.py --records 10000000 --steps 2 > gpurun_out/abl_$a.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 gpurun_out/abl_$a.log; exit 1; fi
  echo "abl=$a $(grep -o '"kernel_ms": {[^}]*}' gpurun_out/abl_$a.log) $(grep -o '"encode_ms": [0-9.]*' gpurun_out/abl_$a.log)"
done
