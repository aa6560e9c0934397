#!/bin/bash
set -e
OUT=${1:-gpurun_out/r03fd2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_decomp.py tests/test_gpu_multiproc.py tests/test_gpu_parity.py tests/test_gpu_graph.py > "$OUT/tests.log" 2>&1
