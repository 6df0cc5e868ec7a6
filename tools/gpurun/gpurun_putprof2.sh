set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pp_tiny" -o put -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload put --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pp_tiny.json 2> gpurun_out/pp.err || { tail gpurun_out/pp.err; exit 1; }
KDB_LZ4_TINY=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pp_notiny" -o put -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload put --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pp_notiny.json 2> gpurun_out/pp.err || { tail gpurun_out/pp.err; exit 1; }
for d in pp_tiny pp_notiny; do echo $d; python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/$d/put_kernel_stats.csv')):
    print('  %-60s %6s %8.4f ms avg %8.3f tot' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6, float(r['TotalDurationNs'])/1e6))
"; done
