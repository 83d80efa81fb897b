#!/bin/bash
# Round 5: SQ instruction / activity counters of k_crc variants (kbench counter mode), one rocprofv3 --pmc pass per set.
# usage: r05_pmc_sq.sh TAG MODE VARIANT   -> gpurun_out/r05pmc/TAG/<set>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
TAG=$1; MODE=$2; V=$3
OUT=$R/gpurun_out/r05pmc/$TAG
mkdir -p "$OUT"
declare -A SETS
SETS[a]="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
SETS[b]="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
SETS[c]="SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_IFETCH SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES SQ_INSTS_SENDMSG"
SETS[d]="SQC_ICACHE_MISSES SQC_ICACHE_HITS"
for k in a b c d; do
  rm -rf "$OUT/$k"
  timeout -s KILL 120 rocprofv3 --pmc ${SETS[$k]} -d "$OUT/$k" -o run --output-format csv -- \
    tools/kbench/kbench $((1 << 30)) $MODE 2 $V > "$OUT/$k.log" 2>&1 || { tail -5 "$OUT/$k.log"; exit 1; }
done
python3 tools/pmc_table.py "k_crc<$V>" "$OUT"/a "$OUT"/b "$OUT"/c "$OUT"/d
