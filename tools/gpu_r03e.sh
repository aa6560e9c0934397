#!/bin/bash
# halo pack/unpack rewrite: decomposed parity tests, then the rank simulation
set -e
OUT=${1:-gpurun_out/r03e}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_decomp.py tests/test_gpu_transport.py -k "decomp or stub or ring1 or part or overlap or ragged or rccl" > "$OUT/tests.log" 2>&1
timeout -k 10 300 python3 tools/rank_sim.py --graph 1 --overlap 0 > "$OUT/rank_g1_ov0.json" 2> "$OUT/rank.err"
timeout -k 10 300 python3 tools/rank_sim.py --graph 1 --overlap 1 --full 0 > "$OUT/rank_g1_ov1.json" 2>> "$OUT/rank.err"
timeout -k 10 300 python3 tools/rank_sim.py --graph 0 --overlap 0 --full 0 > "$OUT/rank_g0_ov0.json" 2>> "$OUT/rank.err"
timeout -k 10 300 python3 tools/rank_sim.py --graph 0 --overlap 1 --full 0 > "$OUT/rank_g0_ov1.json" 2>> "$OUT/rank.err"
