set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc.sh gpurun_out/sq python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-verify --steps 1 --warmup 0 || exit 1
python tools/pmc_summary.py gpurun_out/sq > gpurun_out/sq_summary.txt
cat gpurun_out/sq_summary.txt
