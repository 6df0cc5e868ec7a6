set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out /tmp/lib_dbg; ln -sf $PWD/kingdb_amd/var/var_dbg.so /tmp/lib_dbg/libkdb_lz4.so
for ib in device; do
  for sz in 100; do
    KDB_LZ4_SERVICE_WAVES=1 KDB_LZ4_SVC_INBOX=$ib LD_LIBRARY_PATH=/tmp/lib_dbg timeout -k 10 120 oracle/_ref/kingdb_dropin/bench_compressor $sz 2000 > gpurun_out/dbg_$ib$sz.json 2> gpurun_out/dbg_$ib$sz.err || { echo rc=$?; exit 1; }
    echo "$ib $sz $(cat gpurun_out/dbg_$ib$sz.json)"; grep SVCDBG gpurun_out/dbg_$ib$sz.err | head -4
  done
done
for sz in 100 4096; do
  timeout -k 10 120 oracle/_ref/kingdb_dropin/bench_compressor $sz 4000 > gpurun_out/scalar_$sz.json || { echo rc=$?; exit 1; }
  echo "shipped $sz $(cat gpurun_out/scalar_$sz.json)"
done
