# Rehearsal of the N > 1 bench path on a 1-GPU box: 2 ranks (gloo barrier /
# max-over-ranks, per-rank shards) sharing GPU 0.  Each step bounded; stop at first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
run2() {  # name, port, bench args...
  local name=$1 port=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 "$@" > gpurun_out/r2_$name.json 2> gpurun_out/r2_$name.err \
    || { echo "$name rc=$?"; tail -30 gpurun_out/r2_$name.err; exit 1; }
  cat gpurun_out/r2_$name.json
}
run2 headline 29511 --steps 5 --warmup 2
run2 mixed 29512 --workload mixed --steps 5 --warmup 2
run2 put 29513 --workload put --steps 5 --warmup 2
run2 get 29514 --workload get --steps 5 --warmup 2
echo "== done $(date +%T)"
