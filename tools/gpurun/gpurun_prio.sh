# A/B of KDB_LZ4_BIGPRIO (wave priority of the big-value class launches) on the
# mixed batch, after the parity tests run with it on.  Each step bounded; stop at first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== tests (prio on) $(date +%T)"
KDB_LZ4_BIGPRIO=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/prio_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/prio_tests.log; exit 1; }
tail -1 gpurun_out/prio_tests.log
for r in 1 2 3; do
  for p in 0 1; do
    KDB_LZ4_BIGPRIO=$p timeout -k 10 300 python bench.py --workload mixed --steps 10 --warmup 2 > gpurun_out/prio_m$p.json 2> gpurun_out/prio_m$p.err || { echo "mixed p=$p rc=$?"; tail -20 gpurun_out/prio_m$p.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/prio_m$p.json'));print('mixed prio=$p', d['value'], d['kernels_ms'])"
  done
done
for p in 0 1; do
  KDB_LZ4_BIGPRIO=$p timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/prio_u$p.json 2> gpurun_out/prio_u$p.err || { echo "uniform p=$p rc=$?"; tail -20 gpurun_out/prio_u$p.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/prio_u$p.json'));print('uniform prio=$p', d['value'], d['kernels_ms'])"
done
echo "== done $(date +%T)"
