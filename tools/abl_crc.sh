#!/bin/bash
# k_crc ablation sweep (tools/kbench counter mode, config B): VARIANTS = ABL bit sets of k_crc
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for v in ${VARIANTS:-0 128 256 384 1024 8 4 2 1 0}; do
  timeout -k 10 60 ./tools/kbench/kbench 1073741824 0 10 $v 2>&1 | grep done || exit 1
done
