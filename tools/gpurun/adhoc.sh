set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n26
timeout -k 10 900 python -u -m pytest tests/test_kingdb_dropin.py -x -q -m gpu -k hook --timeout 600 --timeout-method thread > ${O}_hook.log 2>&1 || { tail -30 ${O}_hook.log; exit 1; }
tail -1 ${O}_hook.log
for i in 1 2 3 4 5 6; do
  b=kingdb_hook; d=/tmp/ce_${b}_$i; rm -rf $d; mkdir -p $d; cd $d
  KDB_LZ4_FLUSH_STATS=1 timeout -k 10 120 $GRAFT_REPO_ROOT/oracle/_ref/$b/client_emb > $GRAFT_REPO_ROOT/${O}_ce_$i.txt 2>&1 || { cd $GRAFT_REPO_ROOT; echo "rc=$?"; tail ${O}_ce_$i.txt; exit 1; }
  cd $GRAFT_REPO_ROOT; rm -rf $d
  echo "$i: $(grep -E 'done in' ${O}_ce_$i.txt | head -1) $(grep -oE 'batches [0-9]+|client_stalls.*' ${O}_ce_$i.txt | tr '\n' ' ')"
done
