#!/bin/bash
# wave-state counters (quad-cycles) of k_crc variants (one pass each): where the waves' time goes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r04pmc3
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $*; do
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS -d "$OUT/v${v}" -o run --output-format csv -- \
      ./tools/kbench/kbench $((1 << 30)) ${MODE:-0} 1 $v > "$OUT/v${v}.log" 2>&1 || { tail -5 "$OUT/v${v}.log"; exit 1; }
done
