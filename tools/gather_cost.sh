#!/bin/bash
# Timing-only experiment builds of dyn_tend B with fewer gathered columns (wrong values):
# how much of B's time each gather instruction costs.  Builds into /tmp, then (on the GPU
# box) tools/kbench.py per build with MPAS_LIB.
#   build:  bash tools/gather_cost.sh build      run:  bash tools/gather_cost.sh run OUT
set -e
CS=$(cd "$(dirname "$0")/../mpas-regent_amd/csrc" && pwd)
D=$(cd "$(dirname "$0")/.." && pwd)/abl
if [ "$1" = build ]; then
  mkdir -p "$D"
  for v in "10 8" "6 8" "2 8" "10 4" "10 0"; do
    set -- $v
    o="$D/expt_e$1_a$2"; mkdir -p "$o"
    for f in "$CS"/*.hip "$CS"/*.cpp; do
      b=$(basename "$f"); b=${b%.*}
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -munsafe-fp-atomics \
        -I"$CS/../../include" -I"$CS" -DMPAS_EXPT_EOE=$1 -DMPAS_EXPT_ADV=$2 -c -o "$o/$b.o" "$f" &
    done
    wait
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$D/libmpasdyn_e$1_a$2.so" "$o"/*.o -ldl
    rm -rf "$o"
  done
  exit 0
fi
OUT=${2:-gpurun_out/gcost}
mkdir -p "$OUT"
for so in "$D"/libmpasdyn_e*_a*.so; do
  n=$(basename "$so" .so)
  MPAS_LIB="$so" timeout -k 10 200 python3 tools/kbench.py --rounds 3 --variants "hfuse=0" > "$OUT/$n.json"
done
