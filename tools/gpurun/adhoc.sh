set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n17
timeout -k 10 900 python -u -m pytest tests/test_kingdb_dropin.py -x -q -m gpu -k hook --timeout 600 --timeout-method thread > ${O}_hook.log 2>&1 || { tail -30 ${O}_hook.log; exit 1; }
tail -2 ${O}_hook.log
timeout -k 10 800 python -u tools/write_path_cmp.py --sizes 100 --builds kingdb_hook --repeat 16 --dir /dev/shm --timeout 40 --out ${O}_hang_hunt.json > ${O}_hang_hunt.log 2>&1 || { tail -30 ${O}_hang_hunt.log; exit 1; }
python -c "
import json
rows=json.load(open('${O}_hang_hunt.json'))
print(len(rows),'runs', sum(1 for r in rows if r.get('hung')),'hung')
print([r.get('puts_per_s') for r in rows])
"
