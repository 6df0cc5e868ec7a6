set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n27
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)  nproc: $(nproc)"
for i in 1 2 3 4 5 6; do
  b=kingdb_hook; d=/tmp/ce_${b}_$i; rm -rf $d; mkdir -p $d; cd $d
  t0=$(grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' ')
  KDB_LZ4_FLUSH_STATS=1 timeout -k 10 120 $GRAFT_REPO_ROOT/oracle/_ref/$b/client_emb > $GRAFT_REPO_ROOT/${O}_ce_$i.txt 2>&1 || { cd $GRAFT_REPO_ROOT; echo "rc=$?"; exit 1; }
  t1=$(grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' ')
  cd $GRAFT_REPO_ROOT; rm -rf $d
  echo "$i: $(grep -E 'done in' ${O}_ce_$i.txt | head -1) $(grep -oE 'client_max_gap_ms [0-9.]+' ${O}_ce_$i.txt) | before: $t0 | after: $t1"
done
