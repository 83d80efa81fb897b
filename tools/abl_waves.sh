#!/bin/bash
# k_crc timing of kbench builds with different waves per workgroup (tools/kbench/kbench_w*, -DBCW_CRC_WAVES)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for b in ${BINS:-kbench kbench_w8 kbench_w10}; do
  for v in ${VARIANTS:-0 2 1}; do
    timeout -k 10 60 ./tools/kbench/$b 1073741824 0 10 $v 2>&1 | grep done | sed "s/^/$b /" || exit 1
  done
done
