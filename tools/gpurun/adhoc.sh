set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n22
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > ${O}_quick_$i.json 2> ${O}_quick_$i.err || { tail ${O}_quick_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('${O}_quick_$i.json').read().strip().splitlines()[-1]);print($i, d['value'], d['kernels_ms'], d['roofline']['traffic'])"
done
