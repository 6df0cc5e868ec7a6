set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r03_n11
export PYTHONFAULTHANDLER=1
timeout -s ABRT -k 10 150 python -u bench.py --workload put --values 131072 --steps 2 --warmup 1 --no-cpu-baseline > ${O}_put_small.json 2> ${O}_put_small.err || { echo "put small rc=$?"; grep -v amdgpu.ids ${O}_put_small.err | tail -60; exit 1; }
tail -1 ${O}_put_small.json | cut -c1-300
timeout -s ABRT -k 10 170 python -u bench.py --workload put > ${O}_put.json 2> ${O}_put.err || { echo "put rc=$?"; grep -v amdgpu.ids ${O}_put.err | tail -60; exit 1; }
tail -1 ${O}_put.json | cut -c1-300
timeout -s ABRT -k 10 170 python -u bench.py --workload get > ${O}_get.json 2> ${O}_get.err || { echo "get rc=$?"; grep -v amdgpu.ids ${O}_get.err | tail -60; exit 1; }
tail -1 ${O}_get.json | cut -c1-300
