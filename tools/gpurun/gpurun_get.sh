set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload get > gpurun_out/get.json 2> gpurun_out/get.err || { tail -20 gpurun_out/get.err; exit 1; }
cat gpurun_out/get.json
