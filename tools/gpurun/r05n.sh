set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed_ring.py tests/test_gpu_digests.py tests/test_gpu_fuzz.py -x -v -m gpu --timeout 200 --timeout-method thread > ${O}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 ${O}_tests.log; exit 1; }
tail -2 ${O}_tests.log
bash tools/gpurun/envab.sh $1_ab tune --no-headline --mixed -- KDB_LZ4_DMIXED_ORING2=0 KDB_LZ4_DMIXED_ORING2=1 KDB_LZ4_DMIXED_ORING2=0 KDB_LZ4_DMIXED_ORING2=1 || exit 1
cat gpurun_out/$1_ab.txt
bash tools/gpurun/run.sh $1 bench big readrandom
