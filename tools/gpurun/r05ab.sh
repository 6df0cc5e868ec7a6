# Round-5 A/B session: parity subset on the in-tree build, then alternating
# A/B timings of a baseline variant and the in-tree build (tools/ab.py, digest-gated).
#   bash tools/gpurun/r05ab.sh <tag> <tests|notests> <variant>... 
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; mode=$2; shift 2
O=gpurun_out/$tag
if [ "$mode" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_digests.py tests/test_gpu_service.py tests/test_gpu_hardening.py -x -v -m gpu --timeout 300 --timeout-method thread > ${O}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 ${O}_tests.log; exit 1; }
  tail -3 ${O}_tests.log
fi
for rep in 1 2; do
  for v in "$@"; do
    so=kingdb_amd/var/var_$v.so; [ "$v" = tree ] && so=kingdb_amd/libkdb_lz4.so
    timeout -k 10 200 python tools/ab.py $so --mixed >> ${O}_ab.txt 2>&1 || { echo "ab $v rc=$?"; tail -20 ${O}_ab.txt; exit 1; }
  done
done
cat ${O}_ab.txt
