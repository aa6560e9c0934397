#!/bin/bash
set -e
OUT=${1:-gpurun_out/r03g}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fusedamp or srk3 or dt_zero" tests/test_gpu_main_run.py tests/test_gpu_graph.py tests/test_gpu_bench.py > "$OUT/tests.log" 2>&1
timeout -k 10 400 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 200 python3 bench.py --ncells 2562 --steps 50 --warmup 5 --no-cpu-baseline --traffic off > "$OUT/bench_x1.2562.json" 2>> "$OUT/bench.err"
