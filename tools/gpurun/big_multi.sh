# The big workload line for several library builds (var_<name>.so; tree = in-tree),
# round robin, 2 rounds, with a quick parity pass of each first:
#   big_multi.sh <tag> <name> ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1; shift
lib() { [ "$1" = tree ] && echo "$PWD/kingdb_amd/libkdb_lz4.so" || echo "$PWD/kingdb_amd/var/var_$1.so"; }
for v in "$@"; do
  KDB_LZ4_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 250 --timeout-method thread -k "big or byu32 or fuzz" > ${O}_parity_$v.log 2>&1 || { echo "parity $v rc=$?"; tail -20 ${O}_parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 ${O}_parity_$v.log)"
done
for r in 1 2; do
  for v in "$@"; do
    KDB_LZ4_LIB=$(lib $v) timeout -k 10 300 python bench.py --workload big --no-cpu-baseline --steps 5 --warmup 2 > ${O}_big_$v.$r.json 2> ${O}_big_$v.$r.err || { echo "big $v rc=$?"; tail -5 ${O}_big_$v.$r.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['kernels_ms'])" ${O}_big_$v.$r.json $v
  done
done
