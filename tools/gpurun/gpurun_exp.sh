set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error|assert" gpurun_out/tests.log | head -20; exit 1; }
tail -1 gpurun_out/tests.log
timeout -k 10 300 python bench.py --workload mixed --no-cpu-baseline > gpurun_out/mixed.json 2> gpurun_out/mixed.err || { echo "mixed rc=$?"; tail -5 gpurun_out/mixed.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/mixed.json'));print('mixed',d['value'],d['kernels_ms'])"
for ch in 65536 131072 262144; do
timeout -k 10 300 python bench.py --workload put --no-cpu-baseline --hi-chunk $ch > gpurun_out/put_$ch.json 2> gpurun_out/put_$ch.err || { echo "put rc=$?"; tail -5 gpurun_out/put_$ch.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/put_$ch.json'));print('put $ch',d['value'],d['step_seconds'],d['last_step_host_seconds'])"
done
