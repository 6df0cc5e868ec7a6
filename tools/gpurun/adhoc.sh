set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n18
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_hardening.py -x -q -m gpu --timeout 120 --timeout-method thread > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -2 ${O}_tests.log
for v in mfirst cur mfirst cur mfirst cur; do
  timeout -k 10 300 python tools/ab.py kingdb_amd/var/var_$v.so --mixed --reps 7 --exact-max-in > ${O}_ab_$v.txt 2>&1 || { tail ${O}_ab_$v.txt; exit 1; }
  cat ${O}_ab_$v.txt
done
