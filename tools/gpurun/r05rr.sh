# readrandom through KingDB under service-wave counts (tools/readrandom_cmp.py), plus the service tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py -x -q -m gpu --timeout 200 --timeout-method thread > ${O}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
for w in "$@"; do
  echo "== KDB_LZ4_SERVICE_WAVES=$w"
  KDB_LZ4_SERVICE_WAVES=$w timeout -k 10 600 python -u tools/readrandom_cmp.py --out ${O}_rr_w$w.json > ${O}_rr_w$w.log 2>&1 || { echo "rr rc=$?"; tail -20 ${O}_rr_w$w.log; exit 1; }
  python - ${O}_rr_w$w.log <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        print(f"{d['build']:14s} {d['value_bytes']:5d} B {d['threads']:3d} thr  {d['reads_per_s']/1e3:8.1f} k reads/s")
PY
done
