#!/bin/bash
# LDS bank-conflict attribution of the headline compress kernel (round 3).
#
#   gpurun -- bash tools/gpurun/lds_attr.sh <tag>
#
# Builds (made beforehand on the CPU, tools/build_variants.sh):
#   var_base  the kernel as it is
#   var_dupx  + the two table exchanges issued a second time as reads (-DKDB_ABL_DUP_XCHG)
#   var_dupc  + the candidate word read a second time                 (-DKDB_ABL_DUP_CAND)
# Each build: one rocprofv3 --pmc pass of LDS counters over one headline step,
# then its timing (tools/ab.py, digest-gated).  The extra SQ_LDS_BANK_CONFLICT
# cycles of a duplicate build are the conflict cycles of the access it repeats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
R=$GRAFT_REPO_ROOT
for v in base dupx dupc; do
  export KDB_LZ4_LIB=$R/kingdb_amd/var/var_$v.so
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU \
      SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d "$R/${O}_sq_$v" -o pmc \
      -- python3 "$R/bench.py" --no-cpu-baseline --no-verify --steps 1 --warmup 0 > "${O}_sq_$v.log" 2>&1 \
      || { echo "pmc $v failed"; tail -20 "${O}_sq_$v.log"; exit 1; }
  unset KDB_LZ4_LIB
  timeout -k 10 200 python tools/ab.py kingdb_amd/var/var_$v.so > "${O}_ab_$v.txt" 2>&1 \
      || { echo "ab $v failed"; tail -20 "${O}_ab_$v.txt"; exit 1; }
  cat "${O}_ab_$v.txt"
done
for v in base dupx dupc; do echo "== $v"; python tools/pmc_summary.py "${O}_sq_$v"; done > "${O}_sq.txt" 2>&1
cat "${O}_sq.txt"
