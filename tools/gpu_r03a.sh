#!/bin/bash
# Round-3 first GPU pass: the new / changed GPU tests, then the full suite, then a bench line.
# usage: bash tools/gpu_r03a.sh OUT
set -e
OUT=${1:-gpurun_out/r03a}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_main_run.py tests/test_gpu_jw.py tests/test_gpu_bench.py \
  "tests/test_gpu_decomp.py::test_ring1_rank_without_boundary_edges" > "$OUT/new_tests.log" 2>&1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
