# one GPU session: bench (with cpu baseline) + rocprofv3 kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed $?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "rocprof failed $?"; tail -20 gpurun_out/prof.err; exit 1; }
find gpurun_out/prof -name "*stats*" | head
for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do cat $f; done
