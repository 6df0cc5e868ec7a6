set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_digests.py tests/test_gpu_service.py tests/test_gpu_hardening.py tests/test_gpu_selftest.py tests/test_gpu_mixed_ring.py tests/test_gpu_inplace_window.py -x -v -m gpu --timeout 300 --timeout-method thread > ${O}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 ${O}_tests.log; exit 1; }
tail -3 ${O}_tests.log
AB_ARGS='--uniform 100:943718' bash tools/gpurun/r05d.sh $1 nosq base m1 tree
