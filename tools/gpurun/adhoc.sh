set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n23
for i in 1 2 3 4 5; do
  for b in kingdb_ref kingdb_hook; do
    d=/tmp/ce_${b}_$i; rm -rf $d; mkdir -p $d; cd $d
    timeout -k 10 120 $GRAFT_REPO_ROOT/oracle/_ref/$b/client_emb > $GRAFT_REPO_ROOT/${O}_ce_${b}_$i.txt 2>&1 || { cd $GRAFT_REPO_ROOT; echo "$b $i rc=$?"; tail ${O}_ce_${b}_$i.txt; exit 1; }
    cd $GRAFT_REPO_ROOT; rm -rf $d
    echo "$b $i: $(grep -E 'done in' ${O}_ce_${b}_$i.txt | tr '\n' ' ')"
  done
done
