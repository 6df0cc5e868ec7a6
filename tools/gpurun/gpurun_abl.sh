set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARS:-base occ4 occ6 noemit nogroup nonext}; do
  timeout -k 10 120 python tools/ablate.py kingdb_amd/var/var_$v.so 2>&1 | tee -a gpurun_out/abl.log || exit 1
done
