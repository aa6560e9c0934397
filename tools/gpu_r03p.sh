#!/bin/bash
# transport edge-group sizes: interleaved A/B per build (MPAS_LIB), tredge on vs off
set -e
OUT=${1:-gpurun_out/r03p}
mkdir -p "$OUT"
export TMPDIR=/tmp
for so in abl/libmpasdyn_tre*.so; do
  n=$(basename "$so" .so)
  MPAS_LIB="$so" timeout -k 10 300 python3 tools/kbench.py --rounds 3 --transport --variants "tredge=1" "tredge=0" > "$OUT/$n.json"
done
