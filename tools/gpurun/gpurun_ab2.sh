set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
tail -3 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
KDB_LZ4_BIGGROUP=bins timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "big or mixed or random or scalar" > gpurun_out/tests2.log 2>&1; rc=$?
tail -3 gpurun_out/tests2.log
[ $rc -eq 0 ] || exit $rc
pr() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value'],d.get('kernels_ms'))" $1; }
for g in ballot bins; do
KDB_LZ4_BIGGROUP=$g timeout -k 10 300 python bench.py --workload mixed --no-cpu-baseline > gpurun_out/ab_mixed_$g.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/ab_mixed_$g.json
KDB_LZ4_BIGGROUP=$g timeout -k 10 300 python bench.py --size 65536 --values 32768 --no-cpu-baseline > gpurun_out/ab_64k_$g.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/ab_64k_$g.json
KDB_LZ4_BIGGROUP=$g timeout -k 10 300 python bench.py --size 16384 --values 131072 --no-cpu-baseline > gpurun_out/ab_16k_$g.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/ab_16k_$g.json
KDB_LZ4_BIGGROUP=$g timeout -k 10 300 python bench.py --size 1048576 --values 2048 --no-cpu-baseline > gpurun_out/ab_1m_$g.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
pr gpurun_out/ab_1m_$g.json
done
