#!/bin/bash
# instruction counts + wave states of k_crc slow-path ablations (no emission)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/r04_pmc2.sh 8 65544 458760 8388616 > /dev/null && bash tools/r04_pmc3.sh 8 65544 458760 8388616 > /dev/null
