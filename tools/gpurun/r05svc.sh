# Per-call latency of the resident services under the protocol knobs (same box, interleaved).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1
for rep in 1 2 3; do
  for kv in "KDB_LZ4_SVC_POST=0 KDB_LZ4_SVC_REPLY=0 KDB_LZ4_SVC_PIPE=0" "KDB_LZ4_SVC_PIPE=0" "KDB_LZ4_SVC_PIPE=1"; do
    env $kv timeout -k 10 120 oracle/_ref/kingdb_dropin/bench_compressor 100 4000 > ${O}_x.json || { echo "rc=$?"; exit 1; }
    echo "$kv $(cat ${O}_x.json)" | tee -a ${O}_svc.txt
  done
  timeout -k 10 120 oracle/_ref/kingdb_ref/bench_compressor 100 4000 > ${O}_x.json || exit 1
  echo "reference $(cat ${O}_x.json)" | tee -a ${O}_svc.txt
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_service.py -x -v -s -m gpu --timeout 200 --timeout-method thread > ${O}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 ${O}_tests.log; exit 1; }
tail -2 ${O}_tests.log
