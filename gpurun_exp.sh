set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # label args...
  local label=$1; shift 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > gpurun_out/exp_$label.json 2> gpurun_out/exp_$label.err || { echo "$label failed"; tail gpurun_out/exp_$label.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp_$label.json'));print('$label', d['value'],d['kernels_ms'],d['compress_gibs'],d['decompress_gibs'])"
  grep persistent gpurun_out/exp_$label.err | sort | uniq -c | head -3
}
KDB_LZ4_DEBUG=1 run occ_def
KDB_LZ4_DEBUG=1 KDB_LZ4_PER_CU=8 run occ8
KDB_LZ4_DEBUG=1 KDB_LZ4_PER_CU=6 run occ6
KDB_LZ4_DEBUG=1 KDB_LZ4_PER_CU=4 run occ4
