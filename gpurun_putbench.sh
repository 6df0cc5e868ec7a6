set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload put --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/put.json 2> gpurun_out/put.err || { echo "put failed"; tail -20 gpurun_out/put.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/put.json'));print(d['value'],d['step_seconds'],d['last_step_host_seconds'])"
