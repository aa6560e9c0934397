#!/bin/bash
# whole-library builds under the AMDGPU scheduler strategies (abl/) against the in-tree build
set -e
OUT=${1:-gpurun_out/r03sch}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for so in mpas-regent_amd/mpasdyn/libmpasdyn.so abl/libmpasdyn_silp.so abl/libmpasdyn_smem.so; do
    n=$(basename $so .so)
    timeout -k 10 200 env MPAS_LIB=$so python3 tools/kbench.py --rounds 3 --variants xcd=64 > "$OUT/${n}_$r.json"
  done
done
