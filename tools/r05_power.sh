#!/bin/bash
# Round-5 attribution of k_crc's slow phase: SMU clocks/power sampled (tools/power_trace.py) beside
#  1. kbench seqk: 80 back-to-back launches of a plain HBM stream, of k_crc, of k_crc without emission, of the pipeline
#     (each from idle: 2 s apart);
#  2. bench.py exactly as the driver runs it (--warmup 5), under a rocprofv3 kernel trace;
#  3. tools/trace_probe.py (80 decodes, pause, 80 decodes) under a rocprofv3 kernel trace.
# Results under gpurun_out/r05p/ (summarised by tools/power_align.py, copied into profiles/ by hand).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05p
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
STOP=$OUT/STOP
python3 tools/power_trace.py "$OUT/smi.csv" --seconds 500 --stop-file "$STOP" > "$OUT/smi.log" 2>&1 &
SP=$!
trap 'touch "$STOP"; wait $SP; cat "$OUT/smi.log"' EXIT
sleep 2
KB=tools/kbench/kbench
for v in -1 0 8 -2; do
  echo "== kbench seqk $v $(date +%T)"
  timeout -k 10 120 $KB $((1 << 30)) 0 seqk 80 $v > "$OUT/seqk_$v.log" 2>&1 || { tail -5 "$OUT/seqk_$v.log"; exit 1; }
  grep -E "mark|seqk" "$OUT/seqk_$v.log" | cut -c1-300
  sleep 2
done
echo "== bench (driver command) under kernel trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/bench_w5" -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/bench_w5.log" 2>&1 || { tail -30 "$OUT/bench_w5.log"; exit 1; }
tail -1 "$OUT/bench_w5.log" | cut -c1-300
sleep 2
echo "== trace_probe under kernel trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/probe" -o run --output-format csv -- \
  python3 tools/trace_probe.py torch 80 > "$OUT/probe.log" 2>&1 || { tail -30 "$OUT/probe.log"; exit 1; }
grep mark "$OUT/probe.log"
sleep 2
echo "== bench (driver command) plain $(date +%T)"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/bench_w5_plain.log" 2>&1 || { tail -30 "$OUT/bench_w5_plain.log"; exit 1; }
tail -1 "$OUT/bench_w5_plain.log" | cut -c1-200
echo "== done $(date +%T)"
