#!/bin/bash
# dyn_tend B occupancy caps (MPAS_B_MINW builds in abl/) at x1.2562 and x1.163842
set -e
OUT=${1:-gpurun_out/r03bw}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for so in mpas-regent_amd/mpasdyn/libmpasdyn.so abl/libmpasdyn_bw5.so abl/libmpasdyn_bw8.so; do
    n=$(basename $so .so)
    timeout -k 10 120 env MPAS_LIB=$so python3 tools/abstep.py --ncells 2562 --rounds 4 --steps 20 --variants xcd=64 > "$OUT/s_${n}_$r.json"
    timeout -k 10 200 env MPAS_LIB=$so python3 tools/abstep.py --ncells 163842 --rounds 2 --steps 5 --variants xcd=64 > "$OUT/b_${n}_$r.json"
  done
done
