#!/bin/bash
# Builds variants of libkdb_lz4.so into kingdb_amd/var/var_<name>.so for A/B runs
# (tools/ab.py), e.g.  tools/build_variants.sh tune:-DKDB_LZ4_TUNING  (environment knobs on)
set -e
cd "$(dirname "$0")/../kingdb_amd"
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc"
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}; [ "$flags" = "$v" ] && flags=""
  d=build/var_$name; mkdir -p $d
  for f in csrc/*.hip; do $H $flags -c $f -o $d/$(basename $f .hip).o & done; wait
  for f in csrc/hstable.cc; do /opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -Icsrc -I../include -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -x c++ -c $f -o $d/$(basename $f .cc).o; done
  mkdir -p var && /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/var_$name.so $d/*.o -Wl,-rpath,/opt/rocm/lib
done
