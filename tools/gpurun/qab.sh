# A/B of work-queue layouts (variants built by tools/build_variants.sh with
# -DKDB_LZ4_TUNING) over claim sizes: bash tools/gpurun/qab.sh <tag> <claim_bytes...> -- <variants...>
set -o pipefail
tag=$1; shift
cbs=(); while [ "$1" != "--" ]; do cbs+=("$1"); shift; done; shift
for cb in "${cbs[@]}"; do
  for v in "$@"; do
    echo "== $v claim_bytes=$cb" >> gpurun_out/${tag}.txt
    KDB_LZ4_CLAIM_BYTES=$cb timeout -k 10 150 python tools/ab.py kingdb_amd/var/var_$v.so --mixed --uniform 100:943718 >> gpurun_out/${tag}.txt 2>&1 || exit 1
  done
done
