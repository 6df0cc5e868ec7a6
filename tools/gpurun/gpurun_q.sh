set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
tail -2 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
pr() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value'],d.get('kernels_ms'),d.get('step_seconds'))" $1; }
for q in 1 8; do
KDB_LZ4_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_head_$q.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/b_head_$q.json
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_head.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/b_head.json
timeout -k 10 300 python bench.py --workload put --no-cpu-baseline > gpurun_out/b_put.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/b_put.json
