# Service checks after a protocol change: the service GPU tests, svc_stress,
# hook_mt, and the per-call latencies (bench_compressor), under KDB_LZ4_SVC_INBOX
# =device (default) and =host.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py -x -v -m gpu --timeout 200 --timeout-method thread > ${O}_svc_tests.log 2>&1 || { echo "svc tests rc=$?"; tail -30 ${O}_svc_tests.log; exit 1; }
tail -1 ${O}_svc_tests.log
export KDB_ORACLE_SO=$PWD/oracle/liblz4_oracle.so
for ib in device host; do
  for busy in 0 1; do
    KDB_LZ4_SVC_INBOX=$ib timeout -k 10 200 tests/cpp/svc_stress 8 300 7 $busy > ${O}_ss_$ib$busy.log 2>&1 || { echo "svc_stress $ib $busy rc=$?"; tail -5 ${O}_ss_$ib$busy.log; exit 1; }
    echo "svc_stress inbox=$ib busy=$busy: $(tail -1 ${O}_ss_$ib$busy.log)"
  done
  rm -rf /tmp/hm_db
  KDB_LZ4_SVC_INBOX=$ib timeout -k 10 200 oracle/_ref/kingdb_hook/hook_mt /tmp/hm_db 8 150 > ${O}_hm_$ib.log 2>&1 || { echo "hook_mt $ib rc=$?"; tail -5 ${O}_hm_$ib.log; exit 1; }
  echo "hook_mt inbox=$ib: $(tail -1 ${O}_hm_$ib.log)"
  for sz in 100 4096; do
    KDB_LZ4_SVC_INBOX=$ib timeout -k 10 120 oracle/_ref/kingdb_dropin/bench_compressor $sz 4000 > ${O}_scalar_${ib}_$sz.json || { echo "scalar rc=$?"; exit 1; }
    echo "scalar inbox=$ib $sz: $(cat ${O}_scalar_${ib}_$sz.json)"
  done
done
