#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace stats, encode bench, kbench.
# STEPS: comma-separated subset of tests,smoke,bench,prof,pmc,enc,kbench. Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-tests,smoke,bench,prof,enc}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
run() { echo "== $1 ($(date +%T))"; }
if has tests; then
  run tests
  timeout -k 10 1000 python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi
if has smoke; then
  run smoke
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
  tail -2 "$OUT/smoke.log"
fi
if has bench; then
  run bench
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
  tail -1 "$OUT/bench.log"
fi
if has kbench; then
  run kbench
  timeout -k 10 300 ./tools/kbench/kbench ${KBENCH_ARGS:-} > "$OUT/kbench.log" 2>&1 || { tail -30 "$OUT/kbench.log"; exit 1; }
  cat "$OUT/kbench.log"
fi
if has prof; then
  run prof
  export TMPDIR=/tmp
  rm -rf "$OUT/prof"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --inflight 1 > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 1; }
  find "$OUT/prof" -name "*stats*" | head
fi
if has pmc; then
  run pmc
  export TMPDIR=/tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf "$OUT/pmc_$c"
    timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --inflight 1 > "$OUT/pmc_$c.log" 2>&1 || { tail -30 "$OUT/pmc_$c.log"; exit 1; }
  done
  find "$OUT" -name "*counter_collection*" | head
fi
if has enc; then
  run enc
  export TMPDIR=/tmp
  timeout -k 10 400 python -u tools/bench_encode.py --records ${RECORDS:-10000000} --out "$OUT/encode_bench.json" \
    > "$OUT/benc.log" 2>&1 || { tail -30 "$OUT/benc.log"; exit 1; }
  tail -1 "$OUT/benc.log" | cut -c1-600
  rm -rf "$OUT/prof_enc"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_enc" -o run --output-format csv -- \
    python3 tools/bench_encode.py --records ${RECORDS:-10000000} --steps 3 --no-cpu-baseline --no-index > "$OUT/prof_enc.log" 2>&1 || { tail -30 "$OUT/prof_enc.log"; exit 1; }
  find "$OUT/prof_enc" -name "*stats*" | head
fi
echo "== done ($(date +%T))"
