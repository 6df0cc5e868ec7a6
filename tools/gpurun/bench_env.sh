# One workload line of a library variant under several environment settings:
#   bench_env.sh <tag> <workload> <variant|tree> <VAR=value|-> ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1; W=$2; v=$3; shift 3
lib() { [ "$1" = tree ] && echo "$PWD/kingdb_amd/libkdb_lz4.so" || echo "$PWD/kingdb_amd/var/var_$1.so"; }
i=0
for kv in "$@"; do
  i=$((i+1)); e=$kv; [ "$kv" = "-" ] && e="KDB_NOTHING=0"
  env KDB_LZ4_LIB=$(lib $v) $e timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --steps 5 --warmup 2 > ${O}_$i.json 2> ${O}_$i.err || { echo "$kv rc=$?"; tail -5 ${O}_$i.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['kernels_ms'])" ${O}_$i.json "$kv"
done
