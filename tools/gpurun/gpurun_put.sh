set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|assert" gpurun_out/tests.log | tail -30; exit 1; }
tail -3 gpurun_out/tests.log
