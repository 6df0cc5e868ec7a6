set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/putprof -o put -- python3 $GRAFT_REPO_ROOT/bench.py --workload put --steps 3 --warmup 1 --no-cpu-baseline --put-chunk 131072 > $GRAFT_REPO_ROOT/gpurun_out/putprof.json 2> $GRAFT_REPO_ROOT/gpurun_out/putprof.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/putprof.err; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/putprof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-4 | cut -c1-150
