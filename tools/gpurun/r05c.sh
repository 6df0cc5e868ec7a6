# Round-5 session: parity subset, compress A/B (base variant vs tree), per-call latency.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_digests.py tests/test_gpu_service.py tests/test_gpu_hardening.py -x -v -m gpu --timeout 300 --timeout-method thread > ${O}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 ${O}_tests.log; exit 1; }
tail -3 ${O}_tests.log
for v in base tree base tree; do
  so=kingdb_amd/var/var_$v.so; [ "$v" = tree ] && so=kingdb_amd/libkdb_lz4.so
  timeout -k 10 200 python tools/ab.py $so --mixed >> ${O}_ab.txt 2>&1 || { echo "ab $v rc=$?"; tail -20 ${O}_ab.txt; exit 1; }
done
cat ${O}_ab.txt
for sz in 100 4096; do
  for v in kingdb_ref kingdb_dropin; do
    timeout -k 10 120 oracle/_ref/$v/bench_compressor $sz 2000 > ${O}_scalar_${v}_$sz.json || { echo "scalar $v $sz rc=$?"; exit 1; }
    echo "$v $sz $(cat ${O}_scalar_${v}_$sz.json)"
  done
done
