set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
tail -3 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
pr() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value'],d['kernels_ms'],d['compress_gibs'],d['decompress_gibs'])" $1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_head.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/b_head.json
timeout -k 10 300 python bench.py --workload mixed --no-cpu-baseline > gpurun_out/b_mixed.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/b_mixed.json
KDB_LZ4_NOFORK=1 timeout -k 10 300 python bench.py --workload mixed --no-cpu-baseline > gpurun_out/b_mixed_nofork.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/b_mixed_nofork.json
timeout -k 10 300 python bench.py --size 65536 --values 32768 --no-cpu-baseline > gpurun_out/b_64k.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/b_64k.json
