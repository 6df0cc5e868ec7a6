set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
tail -5 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['kernels_ms'],d['compress_gibs'],d['decompress_gibs'],d['roofline']['frac'],d['roofline'].get('copy_gbs'))"
timeout -k 10 300 python bench.py --workload mixed --no-cpu-baseline > gpurun_out/mixed.json 2> gpurun_out/mixed.err || { tail gpurun_out/mixed.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/mixed.json'));print(d['value'],d['kernels_ms'],d['compress_gibs'],d['decompress_gibs'])"
