#!/bin/bash
# kernel trace of one rank of the 8-way split (stub transport, graph, no overlap)
set -e
OUT=${1:-gpurun_out/r03d}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv -- python3 tools/rank_sim.py --graph 1 --overlap 0 --full 0 --steps 10 > "$OUT/rank.json" 2> "$OUT/rank.err"
