# A/B of one variant build under environment settings:
#   bash tools/gpurun/envab.sh <tag> <variant> <ab.py args...> -- <VAR=value ...>
# (each VAR=value runs tools/ab.py once; "-" runs with nothing set)
set -o pipefail
tag=$1; v=$2; shift 2
args=(); while [ "$1" != "--" ]; do args+=("$1"); shift; done; shift
for kv in "$@"; do
  echo "== $v $kv" >> gpurun_out/${tag}.txt
  if [ "$kv" = "-" ]; then
    timeout -k 10 150 python tools/ab.py kingdb_amd/var/var_$v.so "${args[@]}" >> gpurun_out/${tag}.txt 2>&1 || exit 1
  else
    env $kv timeout -k 10 150 python tools/ab.py kingdb_amd/var/var_$v.so "${args[@]}" >> gpurun_out/${tag}.txt 2>&1 || exit 1
  fi
done
