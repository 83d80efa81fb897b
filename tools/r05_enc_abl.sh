#!/bin/bash
# Round 5: where k_wcopy's time goes -- the config-E encode with BCW_ENC_ABL measurement ablations (4: no source
# copy, 8: no headers / literal bytes, 16: no split-record CRC, 20: neither copy nor CRC). Output gpurun_out/r05abl/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05abl
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
for a in ${ABLS:-0 4 8 16 20}; do
  BCW_ENC_ABL=$a timeout -k 10 300 python3 tools/bench_encode.py --records ${RECORDS:-10000000} --steps 10 --warmup 3 --no-index --no-cpu-baseline > "$OUT/enc_$a.log" 2>&1; rc=$?; [[ $rc -ne 0 && $rc -ne 1 ]] && { tail -20 "$OUT/enc_$a.log"; exit 1; }
  grep "^{" "$OUT/enc_$a.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('abl $a', 'encode_ms', d['encode_ms'], 'writer', d['kernel_ms'].get('k_write'))"
done
