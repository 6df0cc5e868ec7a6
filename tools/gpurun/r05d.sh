# Round-5 session: A/B of variants (tools/ab.py, digest-gated) then SQ counters of the in-tree build.
#   bash tools/gpurun/r05d.sh <tag> <sq|nosq> <variant>...   (variant "tree" = kingdb_amd/libkdb_lz4.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; sq=$2; shift 2
O=gpurun_out/$tag
for rep in 1 2; do
  for v in "$@"; do
    so=kingdb_amd/var/var_$v.so; [ "$v" = tree ] && so=kingdb_amd/libkdb_lz4.so
    timeout -k 10 200 python tools/ab.py $so --mixed ${AB_ARGS:-} >> ${O}_ab.txt 2>&1 || { echo "ab $v rc=$?"; tail -20 ${O}_ab.txt; exit 1; }
  done
done
cat ${O}_ab.txt
if [ "$sq" = sq ]; then
  timeout -k 10 900 bash tools/pmc.sh "${O}_sq" python3 bench.py --no-cpu-baseline --no-host-inclusive --no-verify --steps 1 --warmup 0 || exit 1
  python tools/pmc_summary.py "${O}_sq" > "${O}_sq.txt" && grep -A24 "lz4_compress_kernel<true, true>" "${O}_sq.txt"
fi
