#!/bin/bash
# round-5 evidence run: GPU suite, smoke, bench.py exactly as the driver runs it (with its extras: config C, CPU
# baselines, end-to-end), rocprofv3 kernel stats of the same command, FETCH/WRITE PMC passes. Results under
# gpurun_out/r05/ (copied into profiles/ by hand). STEPS selects a subset.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-tests,smoke,bench,prof,pmc}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  echo "== tests $(date +%T)"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
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
  tail -1 "$OUT/bench.log" > "$OUT/bench.json"; cut -c1-400 "$OUT/bench.json"
fi
if has prof; then
  echo "== prof $(date +%T)"
  rm -rf "$OUT/prof"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras --inflight 1 > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 1; }
  python3 tools/trace_window.py "$OUT/prof" --skip 6 --steps 20 -o "$OUT/prof_timed.json"
fi
if has pmc; then
  echo "== pmc $(date +%T)"
  for c in RDREQ WRITE_SIZE; do
    set_=$c; [[ $c == RDREQ ]] && set_="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
    rm -rf "$OUT/pmc_$c"
    timeout -k 10 300 rocprofv3 --pmc $set_ -d "$OUT/pmc_$c" -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --inflight 1 > "$OUT/pmc_$c.log" 2>&1 || { tail -30 "$OUT/pmc_$c.log"; exit 1; }
  done
  python3 tools/pmc_summary.py --rdreq "$OUT/pmc_RDREQ" --write "$OUT/pmc_WRITE_SIZE" --kernel "k_crc" \
    --seg-bytes 1073743514 --alg-bytes 1090796956 -o "$OUT/k_crc_pmc.json"
fi
echo "== done $(date +%T)"
