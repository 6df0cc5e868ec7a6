# Per-call latency A/B at 100 B only, many rounds (bench_compressor, 8000 calls):
#   svc_ab100.sh <tag> <rounds> <name> <name> ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; shift 2
for v in "$@"; do mkdir -p /tmp/lib_$v && ln -sf $PWD/kingdb_amd/var/var_$v.so /tmp/lib_$v/libkdb_lz4.so; done
for r in $(seq 1 $R); do
  for v in "$@"; do
    LD_LIBRARY_PATH=/tmp/lib_$v timeout -k 10 120 oracle/_ref/kingdb_dropin/bench_compressor 100 8000 > ${O}_$v.$r.json || { echo "$v rc=$?"; exit 1; }
    echo "$v round $r: $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['compress_us'],d['uncompress_us'])" ${O}_$v.$r.json)"
  done
done
