#!/bin/bash
# fused damping on decomposed meshes: the decomposition tests, then one rank's critical path
set -e
OUT=${1:-gpurun_out/r03fd}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_decomp.py tests/test_gpu_multiproc.py tests/test_gpu_transport.py tests/test_gpu_graph.py > "$OUT/tests.log" 2>&1
for o in 0 1; do
  timeout -k 10 300 python3 tools/rank_sim.py --parts 8 --rank 0 --graph 0 --overlap $o > "$OUT/rs_g0_ov$o.json"
  timeout -k 10 300 python3 tools/rank_sim.py --parts 8 --rank 0 --graph 1 --overlap $o > "$OUT/rs_g1_ov$o.json"
done
