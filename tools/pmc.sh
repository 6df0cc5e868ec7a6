#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass; --pmc only with kernel stats,
# never with the sys/runtime trace domains).  Usage (on the GPU box):
#   bash tools/pmc.sh <outdir> <cmd...>
set -o pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d "$out/pass$i" -o pmc -- "$@" > "$out/pass$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/pass$i.log"; exit 1; }
done <<LIST
${PMC_PASSES:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA
SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS SQ_IFETCH SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS}
LIST
echo "pmc passes done: $i"
