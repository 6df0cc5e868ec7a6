set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n14
timeout -k 10 700 python -u tools/write_path_cmp.py --sizes 100 --builds kingdb_hook,kingdb_ref --repeat 3 --dir /dev/shm --timeout 60 --out ${O}_wpath_devshm_100.json > ${O}_wpath_100.log 2>&1 || { tail -30 ${O}_wpath_100.log; exit 1; }
cut -c1-330 ${O}_wpath_100.log
