set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_selftest.py -x -v -s -m gpu --timeout 200 --timeout-method thread > ${O}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 ${O}_tests.log; exit 1; }
tail -3 ${O}_tests.log
for sz in 100 4096; do
  for v in kingdb_ref kingdb_dropin; do
    timeout -k 10 120 oracle/_ref/$v/bench_compressor $sz 4000 > ${O}_scalar_${v}_$sz.json || { echo "scalar $v $sz rc=$?"; exit 1; }
    echo "$v $sz $(cat ${O}_scalar_${v}_$sz.json)"
  done
done
