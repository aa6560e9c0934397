#!/bin/bash
# mesh numbering: 3-D Morton vs cube-face 2-D Hilbert (MPAS_MESH_ORDER), alternating processes
set -e
OUT=${1:-gpurun_out/r03h}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for o in morton hilbert; do
    timeout -k 10 300 env MPAS_MESH_ORDER=$o python3 tools/kbench.py --rounds 3 --variants xcd=64 > "$OUT/kb_${o}_$r.json"
    timeout -k 10 300 env MPAS_MESH_ORDER=$o python3 tools/kbench.py --transport --rounds 2 --variants xcd=64 > "$OUT/kbt_${o}_$r.json"
    timeout -k 10 120 env MPAS_MESH_ORDER=$o python3 tools/abstep.py --ncells 2562 --rounds 4 --steps 20 --variants xcd=64 > "$OUT/s_${o}_$r.json"
  done
done
