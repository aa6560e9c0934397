#!/bin/bash
# hfuse pairs 4-5 (acoustic + solve_vc, solve_e + next stage's dyn_tend A): parity, A/B, trace
set -e
OUT=${1:-gpurun_out/r03q}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fusedamp" tests/test_gpu_main_run.py tests/test_gpu_graph.py > "$OUT/tests.log" 2>&1
timeout -k 10 200 python3 tools/abstep.py --ncells 2562 --steps 20 --rounds 8 --variants "hfuse=1" "hfuse=1,tmedge=1" "hfuse=0" > "$OUT/ab_small.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/small" -o kt --output-format csv -- python3 bench.py --ncells 2562 --steps 20 --warmup 5 --no-cpu-baseline --traffic off > "$OUT/small.json" 2> "$OUT/small.err"
