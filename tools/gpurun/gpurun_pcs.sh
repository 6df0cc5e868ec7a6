set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pcs" -o pcs -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-verify --steps 2 --warmup 1 > gpurun_out/pcs.log 2>&1 || { echo "stochastic rc=$?"; tail -5 gpurun_out/pcs.log; timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pcs" -o pcs -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-verify --steps 2 --warmup 1 > gpurun_out/pcs2.log 2>&1 || { echo "host_trap rc=$?"; tail -5 gpurun_out/pcs2.log; exit 1; }; }
ls -la gpurun_out/pcs/* | head
