set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload put --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/put.json 2> gpurun_out/put.err || { echo "put failed"; tail -20 gpurun_out/put.err; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['step_seconds'],d['last_step_host_seconds'])" gpurun_out/put.json
timeout -k 10 300 python bench.py --workload put --steps 5 --warmup 2 --no-cpu-baseline --hi-chunk 131072 > gpurun_out/put2.json 2> gpurun_out/put.err || { echo "put failed"; tail -20 gpurun_out/put.err; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['step_seconds'],d['last_step_host_seconds'])" gpurun_out/put2.json
