set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n29
for i in 1 2 3 4 5 6 7 8; do
  b=kingdb_hook; d=/tmp/ce_${b}_$i; rm -rf $d; mkdir -p $d; cd $d
  KDB_LZ4_FLUSH_STATS=1 timeout -k 10 120 $GRAFT_REPO_ROOT/oracle/_ref/$b/client_emb > $GRAFT_REPO_ROOT/${O}_ce_$i.txt 2>&1 || { cd $GRAFT_REPO_ROOT; echo "rc=$?"; exit 1; }
  cd $GRAFT_REPO_ROOT; rm -rf $d
  echo "$i: $(grep -E 'done in' ${O}_ce_$i.txt | head -1) | $(grep -oE '(flushes|waits|wait_ms|complete_ms|client_max_gap_ms|max_wait_ms|max_complete_ms|max_between_ms) [0-9.]+' ${O}_ce_$i.txt | tr "\n" " ") $(grep -E lz4_flush_timeline ${O}_ce_$i.txt)"
done
