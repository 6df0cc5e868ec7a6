# Final check of the committed tree with default settings: parity tests, smoke, default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/final_smoke.log; exit 1; }
cat gpurun_out/final_smoke.log
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/final_bench.err; exit 1; }
cat gpurun_out/final_bench.json
echo "== done $(date +%T)"
