set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n9
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_hardening.py tests/test_capi.py -x -q -m gpu --timeout 120 --timeout-method thread > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -2 ${O}_tests.log
for v in lead cur lead cur; do
  timeout -k 10 300 python tools/ab.py kingdb_amd/var/var_$v.so --mixed --reps 7 --exact-max-in > ${O}_ab_$v.txt 2>&1 || { tail ${O}_ab_$v.txt; exit 1; }
  cat ${O}_ab_$v.txt
done
timeout -k 10 600 python bench.py --host-inclusive > ${O}_bench.json 2> ${O}_bench.err || { tail ${O}_bench.err; exit 1; }
python -c "import json;d=json.loads(open('${O}_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['kernels_ms']);h=d['host_inclusive'];print(h['value'],h['compress_gibs'],h['decompress_gibs']);print(json.dumps(h['stall_profile']))"
timeout -k 10 900 python -u -m pytest tests/test_kingdb_dropin.py -x -q -m gpu -k hook --timeout 600 --timeout-method thread > ${O}_hook.log 2>&1 || { tail -30 ${O}_hook.log; exit 1; }
tail -2 ${O}_hook.log
for i in 1 2; do
  for b in kingdb_ref kingdb_hook; do
    d=/tmp/ce_${b}_$i; rm -rf $d; mkdir -p $d; cd $d
    KDB_LZ4_FLUSH_STATS=1 timeout -k 10 120 $GRAFT_REPO_ROOT/oracle/_ref/$b/client_emb > $GRAFT_REPO_ROOT/${O}_ce_${b}_$i.txt 2>&1 || { cd $GRAFT_REPO_ROOT; tail ${O}_ce_${b}_$i.txt; exit 1; }
    cd $GRAFT_REPO_ROOT; rm -rf $d
    echo "$b $i: $(grep -E 'done in|lz4_flush_stats' ${O}_ce_${b}_$i.txt | tr '\n' ' ')"
  done
done
