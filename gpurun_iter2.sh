set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/tests.log 2>&1; rc=$?
tail -3 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
for v in ${VARS}; do
  timeout -k 10 120 python tools/ablate.py kingdb_amd/build/var_$v.so 2>&1 | tee -a gpurun_out/abl.log || exit 1
done
