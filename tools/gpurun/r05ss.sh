set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export KDB_ORACLE_SO=$PWD/oracle/liblz4_oracle.so
for v in "$@"; do
  mkdir -p /tmp/lib_$v && ln -sf $PWD/kingdb_amd/var/var_$v.so /tmp/lib_$v/libkdb_lz4.so
  for busy in 0 1; do
    LD_LIBRARY_PATH=/tmp/lib_$v timeout -k 10 200 tests/cpp/svc_stress 8 300 7 $busy > gpurun_out/r05ss_$v.$busy.log 2>&1; rc=$?
    echo "$v busy=$busy rc=$rc $(tail -1 gpurun_out/r05ss_$v.$busy.log)"; [ $rc -gt 1 ] && exit 1
  done
done
exit 0
