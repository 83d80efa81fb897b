#!/bin/bash
# Round 5: k_wcopy variants (units in flight per lane) -- encode parity tests with the default build, then the config-E
# encode bench with each variant library (BCW_LIB) and the default. Output under gpurun_out/r05enc/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05enc
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_gpu_encode.py}
if [[ "$TESTS" != "none" ]]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
  tail -2 "$OUT/tests.log"
fi
for v in ${VARIANTS:-default}; do
  lib=""
  [[ "$v" != "default" ]] && lib="$R/_var/libbcw_$v.so"
  BCW_LIB=$lib timeout -k 10 300 python3 tools/bench_encode.py --records ${RECORDS:-10000000} --steps 10 --warmup 3 --no-index --no-cpu-baseline > "$OUT/enc_$v.log" 2>&1 || { tail -20 "$OUT/enc_$v.log"; exit 1; }
  tail -1 "$OUT/enc_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 'encode_ms', d['encode_ms'], 'writer', d['kernel_ms'].get('k_write'), 'parity', d['parity'])"
done
