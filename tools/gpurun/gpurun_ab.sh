set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
tail -3 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
pr() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value'],d.get('kernels_ms'))" $1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_bins.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/ab_bins.json
KDB_LZ4_GROUP=ballot timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_ballot.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/ab_ballot.json
timeout -k 10 300 python bench.py --size 100 --values 8388608 --no-cpu-baseline > gpurun_out/ab_100.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/ab_100.json
timeout -k 10 300 python bench.py --workload mixed --no-cpu-baseline > gpurun_out/ab_mixed.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/ab_mixed.json
