set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n19
for v in nozero cur nozero cur; do
  timeout -k 10 300 python tools/ab.py kingdb_amd/var/var_$v.so --no-headline --mixed --reps 5 --uniform 100:943718 --uniform 4096:94372 > ${O}_ab_$v.txt 2>&1 || { tail ${O}_ab_$v.txt; exit 1; }
  cat ${O}_ab_$v.txt
done
