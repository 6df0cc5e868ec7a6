# Round-1 GPU session: parity tests, smoke, bench (+host-inclusive), rocprofv3
# kernel stats, PMC traffic passes, mixed + put workloads.  Each GPU step bounded; stop at first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
step bench
timeout -k 10 600 python bench.py --host-inclusive > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
step mixed
timeout -k 10 300 python bench.py --workload mixed > gpurun_out/mixed.json 2> gpurun_out/mixed.err || { echo "mixed rc=$?"; tail -20 gpurun_out/mixed.err; exit 1; }
cat gpurun_out/mixed.json
step put
timeout -k 10 400 python bench.py --workload put > gpurun_out/put.json 2> gpurun_out/put.err || { echo "put rc=$?"; tail -20 gpurun_out/put.err; exit 1; }
cat gpurun_out/put.json
step get
timeout -k 10 300 python bench.py --workload get > gpurun_out/get.json 2> gpurun_out/get.err || { echo "get rc=$?"; tail -20 gpurun_out/get.err; exit 1; }
cat gpurun_out/get.json
step rocprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "rocprof rc=$?"; tail -20 gpurun_out/prof.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_mixed" -o mixed -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload mixed --steps 3 --warmup 1 > gpurun_out/prof_mixed.json 2> gpurun_out/prof_mixed.err || { echo "rocprof mixed rc=$?"; tail -20 gpurun_out/prof_mixed.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_put" -o put -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload put --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/prof_put.json 2> gpurun_out/prof_put.err || { echo "rocprof put rc=$?"; tail -20 gpurun_out/prof_put.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_get" -o get -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload get --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/prof_get.json 2> gpurun_out/prof_get.err || { echo "rocprof get rc=$?"; tail -20 gpurun_out/prof_get.err; exit 1; }
step pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c" -o pmc -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-verify --steps 1 --warmup 0 > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c rc=$?"; tail -20 gpurun_out/pmc_$c.log; exit 1; }
done
python tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE 1048576 4096 gpurun_out/pmc_traffic.json
step sq
bash tools/pmc.sh gpurun_out/sq python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-verify --steps 1 --warmup 0 || exit 1
python tools/pmc_summary.py gpurun_out/sq > gpurun_out/sq_summary.txt
step done
