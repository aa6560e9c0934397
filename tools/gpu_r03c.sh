#!/bin/bash
# stub-transport rank simulation (per-rank critical path of the 8-GPU run) + its tests
set -e
OUT=${1:-gpurun_out/r03c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_decomp.py -k "stub or ring1 or part_file" > "$OUT/tests.log" 2>&1
timeout -k 10 300 python3 tools/rank_sim.py --graph 0 > "$OUT/rank_g0.json" 2> "$OUT/rank.err"
timeout -k 10 300 python3 tools/rank_sim.py --graph 1 --full 0 > "$OUT/rank_g1.json" 2>> "$OUT/rank.err"
timeout -k 10 300 python3 tools/rank_sim.py --graph 1 --overlap 0 --full 0 > "$OUT/rank_g1_ov0.json" 2>> "$OUT/rank.err"
timeout -k 10 300 python3 tools/rank_sim.py --graph 0 --overlap 0 --full 0 > "$OUT/rank_g0_ov0.json" 2>> "$OUT/rank.err"
