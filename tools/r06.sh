#!/bin/bash
# Round-6 GPU runs (one gpurun call): STEPS picks from
#   tests   the -m gpu suite (TESTS selects files, default the whole suite; PYK a -k expression)
#   smoke   __graft_entry__.smoke()
#   bench   bench.py exactly as the driver runs it (config B, --warmup 5 --steps 20)
#   kb      tools/kbench default mode on config B and C (pipeline and per-kernel times, k_chase phase stamps)
#   cmp     tools/kbench k_crc variants (VARIANTS) interleaved, config B and C, in-kernel clock
#   xbal    tools/kbench pipelines with the per-XCD split on / off (config B and C)
#   prof    rocprofv3 kernel trace of the driver's bench command + the timed-window summary
#   pmc     HBM read (TCC_EA0_RDREQ_*) and WRITE_SIZE passes of k_crc (KERNEL) on config B
# Output under gpurun_out/$TAG/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${TAG:-r06}
OUT=$R/gpurun_out/$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-bench}
TESTS=${TESTS:-tests}
VARIANTS=${VARIANTS:-0 8}
KERNEL=${KERNEL:-k_crc}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  echo "== tests $(date +%T)"
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu ${PYK:+-k "$PYK"} -x -v --timeout 150 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -1 "$OUT/gpu_tests.log"
fi
if has smoke; then
  echo "== smoke $(date +%T)"
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
if has bench; then
  echo "== bench $(date +%T)"
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
  tail -1 "$OUT/bench.log" > "$OUT/bench.json"; cut -c1-600 "$OUT/bench.json"
fi
if has kb; then
  for m in 0 1; do
    echo "== kbench config $m $(date +%T)"
    timeout -k 10 300 tools/kbench/kbench $((1 << 30)) $m > "$OUT/kb_$m.log" 2>&1 || { tail -5 "$OUT/kb_$m.log"; exit 1; }
    grep -E "pipeline|k_chase|k_crc|stream" "$OUT/kb_$m.log" | head -20
  done
fi
if has cmp; then
  for m in 0 1; do
    echo "== kbench cmp config $m $(date +%T)"
    KB_CLOCK=1 timeout -k 10 300 tools/kbench/kbench $((1 << 30)) $m cmp $VARIANTS > "$OUT/cmp_$m.log" 2>&1 || { tail -5 "$OUT/cmp_$m.log"; exit 1; }
    grep -E -A1 "k_crc<" "$OUT/cmp_$m.log"
  done
fi
if has xbal; then
  for m in 0 1; do
    echo "== kbench xbal config $m $(date +%T)"
    timeout -k 10 300 tools/kbench/kbench $((1 << 30)) $m xbal > "$OUT/xbal_$m.log" 2>&1 || { tail -5 "$OUT/xbal_$m.log"; exit 1; }
    grep -E "xbal" "$OUT/xbal_$m.log"
  done
fi
if has prof; then
  echo "== prof $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras --inflight 1 > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 1; }
  python3 tools/trace_window.py "$OUT/prof" --skip 6 --steps 20 -o "$OUT/prof_timed.json" && cat "$OUT/prof_timed.json" | head -40
fi
if has pmc; then
  echo "== pmc $(date +%T)"
  for c in RDREQ WRITE_SIZE; do
    set_=$c; [[ $c == RDREQ ]] && set_="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
    timeout -s KILL 300 rocprofv3 --pmc $set_ -d "$OUT/pmc_$c" -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --inflight 1 > "$OUT/pmc_$c.log" 2>&1 || { tail -30 "$OUT/pmc_$c.log"; exit 1; }
  done
  python3 tools/pmc_summary.py --rdreq "$OUT/pmc_RDREQ" --write "$OUT/pmc_WRITE_SIZE" --kernel "$KERNEL" \
    --seg-bytes 1073743514 --alg-bytes ${ALG_BYTES:-1090796956} -o "$OUT/k_crc_pmc.json" && cat "$OUT/k_crc_pmc.json"
fi
echo "== done $(date +%T)"
