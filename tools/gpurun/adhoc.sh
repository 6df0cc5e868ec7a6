set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n21
for v in vbase ilp clause bias0 vbase ilp clause bias0; do
  timeout -k 10 300 python tools/ab.py kingdb_amd/var/var_$v.so --mixed --reps 5 --exact-max-in > ${O}_ab_$v.txt 2>&1 || { tail ${O}_ab_$v.txt; exit 1; }
  cat ${O}_ab_$v.txt
done
