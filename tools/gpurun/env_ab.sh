# Parity tests, then one workload line under two settings of an environment knob,
# alternating:  env_ab.sh <tag> <workload> <VAR> <value_a> <value_b>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/$1; W=$2; V=$3
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 300 --timeout-method thread > ${O}_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 ${O}_parity.log; exit 1; }
tail -1 ${O}_parity.log
for r in 1 2; do
  for x in $4 $5; do
    env $V=$x timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --steps 5 --warmup 2 > ${O}_${W}_$x.$r.json 2> ${O}_${W}_$x.$r.err || { echo "$W $V=$x rc=$?"; tail -5 ${O}_${W}_$x.$r.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['kernels_ms'])" ${O}_${W}_$x.$r.json "$V=$x"
  done
done
