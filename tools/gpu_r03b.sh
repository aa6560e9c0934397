#!/bin/bash
# fused damping: the new parity tests, the whole-step / decomposed / bounds suites, a bench line
set -e
OUT=${1:-gpurun_out/r03b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fusedamp or srk3 or dt_zero" tests/test_gpu_main_run.py > "$OUT/fused_tests.log" 2>&1
timeout -k 10 400 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1
