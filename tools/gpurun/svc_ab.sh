# A/B of per-call latency (bench_compressor through the drop-in) between library
# builds kingdb_amd/var/var_<name>.so, alternating, 3 rounds:
#   svc_ab.sh <tag> <name> <name> ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1; shift
for v in "$@"; do mkdir -p /tmp/lib_$v && ln -sf $PWD/kingdb_amd/var/var_$v.so /tmp/lib_$v/libkdb_lz4.so; done
for r in 1 2 3; do
  for v in "$@"; do
    for sz in 100 4096; do
      LD_LIBRARY_PATH=/tmp/lib_$v env ${NOVERIFY:+KDB_BENCH_NOVERIFY=1} timeout -k 10 120 oracle/_ref/kingdb_dropin/bench_compressor $sz 4000 > ${O}_$v.$sz.$r.json || { echo "$v rc=$?"; exit 1; }
      echo "$v $sz round $r: $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['compress_us'],d['uncompress_us'])" ${O}_$v.$sz.$r.json)"
    done
  done
done
