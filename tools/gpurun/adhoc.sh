set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_selftest.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03_n2_tests.log 2>&1 || { tail -30 gpurun_out/r03_n2_tests.log; exit 1; }
tail -2 gpurun_out/r03_n2_tests.log
timeout -k 10 300 python tools/ab.py kingdb_amd/libkdb_lz4.so --no-headline --reps 3 --uniform 65536:128 --uniform 65536:256 --uniform 65536:512 --uniform 65536:768 --uniform 65536:1024 --uniform 65536:1536 --uniform 65536:2560 --uniform 16384:2560 --uniform 16384:1024 --uniform 16384:512 > gpurun_out/r03_n2_curve.txt 2>&1 || { tail gpurun_out/r03_n2_curve.txt; exit 1; }
cat gpurun_out/r03_n2_curve.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03_n2_quick.json 2> gpurun_out/r03_n2_quick.err || exit 1
tail -1 gpurun_out/r03_n2_quick.json | cut -c1-400
