set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1; shift
for spec in "$@"; do
  v=${spec%%@*}; envs=${spec#*@}; [ "$envs" = "$spec" ] && envs="KDB_LZ4_X=1"
  mkdir -p /tmp/lib_$v && ln -sf $PWD/kingdb_amd/var/var_$v.so /tmp/lib_$v/libkdb_lz4.so
  for i in 1 2 3; do
    rm -rf /tmp/hm_db
    env ${envs//,/ } LD_LIBRARY_PATH=/tmp/lib_$v KDB_LZ4_SERVICE_WAVES=1 KDB_LZ4_READ_BATCH=64 timeout -k 10 120 oracle/_ref/kingdb_hook/hook_mt /tmp/hm_db 8 150 > ${O}_$v.$i.log 2>&1; rc=$?
    echo "$spec run $i rc=$rc $(tail -1 ${O}_$v.$i.log)"
    [ $rc -gt 1 ] && exit 1
  done
done
exit 0
