set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n20
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -v -m gpu --timeout 300 --timeout-method thread > ${O}_fuzz.log 2>&1 || { tail -40 ${O}_fuzz.log; exit 1; }
tail -4 ${O}_fuzz.log
