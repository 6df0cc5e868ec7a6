# Big-part (1 MiB, byU32) parity tests, then the big workload line for two library
# builds, alternating:  big_ab.sh <tag> <var_a> <var_b>   (tree = the in-tree library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1; A=$2; B=$3
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 ${O}_parity.log; exit 1; }
tail -1 ${O}_parity.log
lib() { [ "$1" = tree ] && echo "$PWD/kingdb_amd/libkdb_lz4.so" || echo "$PWD/kingdb_amd/var/var_$1.so"; }
for r in 1 2; do
  for v in $A $B; do
    KDB_LZ4_LIB=$(lib $v) timeout -k 10 300 python bench.py --workload big --no-cpu-baseline --steps 5 --warmup 2 > ${O}_big_$v.$r.json 2> ${O}_big_$v.$r.err || { echo "big $v rc=$?"; tail -5 ${O}_big_$v.$r.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['kernels_ms'])" ${O}_big_$v.$r.json $v
  done
done
