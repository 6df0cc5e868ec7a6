set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n16
export KDB_LZ4_FLUSH_WATCH=5
timeout -k 10 800 python -u tools/write_path_cmp.py --sizes 100,4096 --builds kingdb_hook --repeat 12 --dir /dev/shm --timeout 40 --out ${O}_hang_hunt.json > ${O}_hang_hunt.log 2>&1 || { tail -30 ${O}_hang_hunt.log; exit 1; }
python -c "
import json
rows=json.load(open('${O}_hang_hunt.json'))
print(len(rows),'runs', sum(1 for r in rows if r.get('hung')),'hung')
for r in rows:
    print(r['workload'][:24], r.get('hung'), r.get('puts_per_s'), r.get('puts_per_s_with_close'))
    if r.get('hung'): print(r['stderr_tail'][-800:])
"
