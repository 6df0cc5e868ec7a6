set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_write_path.py -m gpu > gpurun_out/wp_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/wp_tests.log; exit 1; }
tail -2 gpurun_out/wp_tests.log
for mode in "" "--put-host-copy"; do
timeout -k 10 300 python bench.py --workload put --steps 5 --warmup 2 --no-cpu-baseline $mode > gpurun_out/put$mode.json 2> gpurun_out/put$mode.err || { echo "put failed"; tail -20 gpurun_out/put$mode.err; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value'],d['step_seconds'],d['last_step_host_seconds'])" gpurun_out/put$mode.json
done
