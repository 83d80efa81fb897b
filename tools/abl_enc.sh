#!/bin/bash
# Encode ablations (measurement only): BCW_ENC_ABL bits 4 = k_wcopy without the source copy, 8 = without
# literal / header stores, 16 = without the split-record CRC. Runs with ablations fail parity by design.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for a in ${ABLS:-0 4}; do
  BCW_ENC_ABL=$a timeout -k 10 200 python3 tools/bench_encode.py --records ${RECORDS:-10000000} --steps 3 > gpurun_out/abl_$a.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $a -eq 0 ]; then tail -5 gpurun_out/abl_$a.log; exit 1; fi
  if [ $rc -gt 1 ]; then tail -5 gpurun_out/abl_$a.log; exit 1; fi
  echo "abl $a: $(grep '^{' gpurun_out/abl_$a.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["encode_ms"], d["kernel_ms"], d["parity"])')"
done
