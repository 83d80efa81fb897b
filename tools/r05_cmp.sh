#!/bin/bash
# Round 5: kbench k_crc variants interleaved in one process, with the in-kernel clock (cycles = ms x MHz).
# usage: r05_cmp.sh TAG MODE VARIANTS...   (MODE 0: config B, 1: config C)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; MODE=$2; shift 2
OUT=$R/gpurun_out/r05cmp
mkdir -p "$OUT"
KB_CLOCK=1 timeout -k 10 300 tools/kbench/kbench $((1 << 30)) $MODE cmp "$@" > "$OUT/$TAG.log" 2>&1 || { tail -5 "$OUT/$TAG.log"; exit 1; }
grep -E "k_crc<|seg " "$OUT/$TAG.log"
