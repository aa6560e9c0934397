#!/bin/bash
# Experiment builds of libmpasdyn with preprocessor overrides, into abl/ (git-ignored, sent
# to the GPU box), for interleaved A/B with MPAS_LIB:
#   bash tools/expt_builds.sh NAME "-DX=1 -DY=2" [NAME2 "..."] ...
set -e
CS=$(cd "$(dirname "$0")/../mpas-regent_amd/csrc" && pwd)
D=$(cd "$(dirname "$0")/.." && pwd)/abl
mkdir -p "$D"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  o="$D/obj_$name"; mkdir -p "$o"
  for f in "$CS"/*.hip "$CS"/*.cpp; do
    b=$(basename "$f"); b=${b%.*}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -munsafe-fp-atomics \
      -I"$CS/../../include" -I"$CS" $defs -c -o "$o/$b.o" "$f" 2>/dev/null &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$D/libmpasdyn_$name.so" "$o"/*.o -ldl
  rm -rf "$o"
done
