# per-size kernel rates (bounded steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "100 8388608" "1024 1048576" "16384 131072" "65536 32768"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --size $1 --values $2 --steps 3 --warmup 1 > gpurun_out/size_$1.json 2> gpurun_out/size_$1.err || { echo "size $1 failed"; tail gpurun_out/size_$1.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/size_$1.json'));print($1, d['value'],d['kernels_ms'],d['compress_gibs'],d['decompress_gibs'])"
done
