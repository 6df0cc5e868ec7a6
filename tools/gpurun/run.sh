#!/bin/bash
# One parametrised GPU-box session (replaces the round-1 ad-hoc scripts).
#
#   gpurun --timeout 1200 -- bash tools/gpurun/run.sh <tag> <step> [<step> ...]
#
# Steps (run in the order given, each under its own time limit; the session
# stops at the first failure and starts nothing more on the GPU):
#   tests      pytest -m gpu
#   parity     the codec parity test files only
#   smoke      __graft_entry__.smoke()
#   bench      the headline line (bench.py, host-inclusive rate + CPU baseline)
#   quick      the headline line without the CPU baseline / host-inclusive legs
#   mixed put get   the other BASELINE workloads (bench.py --workload ...)
#   prof       rocprofv3 --kernel-trace --stats of the headline bench
#   profmixed profput profget   the same for the other workloads
#   pmc        FETCH_SIZE / WRITE_SIZE passes of the headline -> pmc_traffic.json
#   pmcmixed   the same for the mixed batch; pmcbig: for the 1 MiB parts
#   pmcu:<size>:<values>  the same for a uniform batch of other sizes
#   sq         SQ counter passes of the headline (tools/pmc.sh); sqbig: of the big workload
#   profbig    rocprofv3 --kernel-trace --stats of the big workload
#   dropin     KingDB's unit tests built against the drop-in (tests/test_kingdb_dropin.py)
#   dropinfull the same with the whole test_db and client_emb (KDB_DROPIN_FULL=1)
#   hook       the flush-hook build's tests only (test_kingdb_dropin.py -k hook)
#   wpath      KingDB's write path (kdb_db) with the reference codec, the drop-in and
#              the flush hook, 1 M x 100 B + 128 Ki x 4 KiB, on /tmp and on /dev/shm
#   readrandom db_bench readrandom through KingDB (reference codec, drop-in, hook; 1 and 16 threads)
#   rehearse2  the four bench workloads under torch.distributed.run with 2 ranks on this
#              1-GPU box (ranks share the device): the N > 1 path end to end, not scaling
#   scalar     per-call latency of CompressorLZ4::Compress/Uncompress, drop-in vs reference
#   ab:<NAME>=<VAL>  the quick headline line with one environment knob set
#   var:<name> A/B of kingdb_amd/var/var_<name>.so (tools/ab.py, digest-gated)
# Outputs land in gpurun_out/<tag>_*.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
O=gpurun_out/$tag
R=$GRAFT_REPO_ROOT
say() { echo "== $tag $1 $(date +%T)"; }
fail() { echo "$1 rc=$2"; tail -30 "$3"; exit 1; }
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['metric'],d['value'],d.get('kernels_ms'),d.get('roofline',{}).get('frac'))" "$1"; }
prof() {  # prof <name> <bench args...>
  local n=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/${O}_prof_$n" -o "$n" -- python3 "$R/bench.py" "$@" > "${O}_prof_$n.json" 2> "${O}_prof_$n.err" || fail "prof $n" $? "${O}_prof_$n.err"
  line "${O}_prof_$n.json"
}
pmc() {  # pmc <name> <n_values> <size> <bench args...>
  local n=$1 nv=$2 sz=$3; shift 3
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$R/${O}_pmc_${n}_$c" -o pmc -- python3 "$R/bench.py" --no-cpu-baseline --no-host-inclusive --no-verify --steps 1 --warmup 0 "$@" > "${O}_pmc_${n}_$c.log" 2>&1 || fail "pmc $n $c" $? "${O}_pmc_${n}_$c.log"
  done
  python tools/pmc_traffic.py "${O}_pmc_${n}_FETCH_SIZE" "${O}_pmc_${n}_WRITE_SIZE" "$nv" "$sz" "${O}_pmc_traffic_$n.json" || exit 1
  cat "${O}_pmc_traffic_$n.json"
}
for s in "$@"; do
  say "$s"
  case $s in
    tests)
      timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --durations=25 --timeout 300 --timeout-method thread > "${O}_tests.log" 2>&1 || fail tests $? "${O}_tests.log"
      tail -2 "${O}_tests.log" ;;
    parity)   # the codec parity files only (compress/decompress kernels)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_fuzz.py tests/test_gpu_batch_emit.py tests/test_gpu_inplace_window.py tests/test_gpu_mixed_ring.py tests/test_gpu_hardening.py -x -v -m gpu --timeout 200 --timeout-method thread > "${O}_parity.log" 2>&1 || fail parity $? "${O}_parity.log"
      tail -2 "${O}_parity.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "${O}_smoke.log" 2>&1 || fail smoke $? "${O}_smoke.log"
      cat "${O}_smoke.log" ;;
    bench)
      timeout -k 10 600 python bench.py --host-inclusive > "${O}_bench.json" 2> "${O}_bench.err" || fail bench $? "${O}_bench.err"
      cat "${O}_bench.json" ;;
    quick)
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive > "${O}_quick.json" 2> "${O}_quick.err" || fail quick $? "${O}_quick.err"
      line "${O}_quick.json" ;;
    mixed|put|get|big)
      timeout -k 10 500 python bench.py --workload $s > "${O}_$s.json" 2> "${O}_$s.err" || fail $s $? "${O}_$s.err"
      cat "${O}_$s.json" ;;
    prof) prof bench --no-cpu-baseline --no-host-inclusive --steps 5 --warmup 1 ;;
    profmixed) prof mixed --workload mixed --no-cpu-baseline --steps 3 --warmup 1 ;;
    profput) prof put --workload put --no-cpu-baseline --steps 3 --warmup 1 ;;
    profget) prof get --workload get --no-cpu-baseline --steps 3 --warmup 1 ;;
    profbig) prof big --workload big --no-cpu-baseline --steps 3 --warmup 1 ;;
    pmc) pmc bench 1048576 4096 ;;
    pmcmixed) pmc mixed 1048576 mixed --workload mixed ;;
    pmcbig) pmc big 2560 1048576 --workload big ;;
    pmcu:*)   # pmcu:<size>:<values> -- FETCH/WRITE passes of a uniform batch
      a=${s#pmcu:}; sz=${a%%:*}; nv=${a#*:}
      pmc u${sz} $nv $sz --size $sz --values $nv ;;
    sq)
      timeout -k 10 900 bash tools/pmc.sh "${O}_sq" python3 "$R/bench.py" --no-cpu-baseline --no-host-inclusive --no-verify --steps 1 --warmup 0 || exit 1
      python tools/pmc_summary.py "${O}_sq" > "${O}_sq.txt" && cat "${O}_sq.txt" ;;
    sqbig)
      timeout -k 10 900 bash tools/pmc.sh "${O}_sqbig" python3 "$R/bench.py" --workload big --no-cpu-baseline --no-verify --steps 1 --warmup 0 || exit 1
      python tools/pmc_summary.py "${O}_sqbig" > "${O}_sqbig.txt" && cat "${O}_sqbig.txt" ;;
    dropin|dropinfull)
      [ $s = dropinfull ] && export KDB_DROPIN_FULL=1
      timeout -k 10 1100 python -u -m pytest tests/test_kingdb_dropin.py -x -v -s -m gpu --durations=0 --timeout 1000 --timeout-method thread > "${O}_$s.log" 2>&1 || fail $s $? "${O}_$s.log"
      grep -E "PASSED|FAILED|passed|failed|done in|count items|s call" "${O}_$s.log" | tail -30
      unset KDB_DROPIN_FULL ;;
    hook)
      timeout -k 10 900 python -u -m pytest tests/test_kingdb_dropin.py -x -v -s -m gpu -k hook --timeout 600 --timeout-method thread > "${O}_hook.log" 2>&1 || fail hook $? "${O}_hook.log"
      grep -E "PASSED|FAILED|passed|failed" "${O}_hook.log" | tail -30 ;;
    wpath)
      for d in /tmp /dev/shm; do
        timeout -k 10 900 python -u tools/write_path_cmp.py --ceiling --dir $d --out "${O}_wpath_${d//\//_}.json" > "${O}_wpath.log" 2>&1 || fail wpath $? "${O}_wpath.log"
        cat "${O}_wpath.log"
      done ;;
    rehearse2)
      port=29511
      for w in uniform mixed put get; do
        port=$((port+1))
        timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --workload $w --no-cpu-baseline > "${O}_rehearse2_$w.json" 2> "${O}_rehearse2_$w.err" || fail "rehearse2 $w" $? "${O}_rehearse2_$w.err"
        line "${O}_rehearse2_$w.json"
      done ;;
    readrandom)   # db_bench readrandom through KingDB: reference codec, drop-in, hook; 1 and 16 threads
      timeout -k 10 900 python -u tools/readrandom_cmp.py --out "${O}_readrandom.json" > "${O}_readrandom.log" 2>&1 || fail readrandom $? "${O}_readrandom.log"
      cat "${O}_readrandom.log" ;;
    scalar)   # per-call latency of CompressorLZ4, drop-in (GPU) vs reference codec (CPU)
      for sz in 100 4096 65536; do
        for v in kingdb_ref kingdb_dropin; do
          timeout -k 10 300 oracle/_ref/$v/bench_compressor $sz 2000 > "${O}_scalar_${v}_$sz.json" || fail "scalar $v $sz" $? "${O}_scalar_${v}_$sz.json"
          echo "$v $(cat ${O}_scalar_${v}_$sz.json)"
        done
      done ;;
    var:*)    # A/B of a library build: kingdb_amd/var/var_<name>.so (tools/ab.py: timing + digest gate)
      v=${s#var:}
      timeout -k 10 300 python tools/ab.py kingdb_amd/var/var_$v.so --mixed > "${O}_var_$v.txt" 2>&1 || fail "var $v" $? "${O}_var_$v.txt"
      cat "${O}_var_$v.txt" ;;
    ab:*)
      kv=${s#ab:}
      env "$kv" timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive > "${O}_ab_${kv}.json" 2> "${O}_ab.err" || fail "ab $kv" $? "${O}_ab.err"
      line "${O}_ab_${kv}.json" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
say done
