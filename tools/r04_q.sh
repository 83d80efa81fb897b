#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of k_crc variants in kbench: full, no emission, emission only (is the x2 correction right
# for the emission's narrow reads?)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r04q
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 0 8 32768; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c -d "$OUT/v${v}_$c" -o run --output-format csv -- \
      ./tools/kbench/kbench $((1 << 30)) 0 3 $v > "$OUT/v${v}_$c.log" 2>&1 || { tail -5 "$OUT/v${v}_$c.log"; exit 1; }
  done
done
