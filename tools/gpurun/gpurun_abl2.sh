set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in kingdb_amd/libkdb_lz4.so kingdb_amd/var/var_pfoff.so kingdb_amd/var/var_pf512.so kingdb_amd/var/var_pf256x2.so kingdb_amd/var/var_pf1024.so kingdb_amd/var/var_pf256x4.so; do
  echo -n "$v 64K: "; timeout -k 10 120 python tools/ablate.py $v 32768 65536 || exit 1
  echo -n "$v 16K: "; timeout -k 10 120 python tools/ablate.py $v 131072 16384 || exit 1
done
