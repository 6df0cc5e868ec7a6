set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
run() {  # label args...
  local label=$1; shift 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > gpurun_out/exp_$label.json 2> gpurun_out/exp_$label.err || { echo "$label failed"; tail gpurun_out/exp_$label.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp_$label.json'));print('$label', d['value'],d['kernels_ms'],d['compress_gibs'],d['decompress_gibs'],d['config']['raw_bytes_per_gpu'])"
}
run mixed --workload mixed
run u4k
KDB_LZ4_MID=lds run lds8k --size 8192 --values 524288
