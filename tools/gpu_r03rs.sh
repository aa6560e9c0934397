#!/bin/bash
# one rank of the 8-way split (Hilbert numbering), stub transport, graph / overlap variants,
# the rank with the largest ghost share too
set -e
OUT=${1:-gpurun_out/r03rs}
mkdir -p "$OUT"
export TMPDIR=/tmp
for g in 0 1; do for o in 0 1; do
  timeout -k 10 300 python3 tools/rank_sim.py --parts 8 --rank 0 --graph $g --overlap $o > "$OUT/rs_r0_g${g}_ov${o}.json"
done; done
timeout -k 10 300 python3 tools/rank_sim.py --parts 8 --rank 1 --graph 0 --overlap 1 > "$OUT/rs_r1_g0_ov1.json"
