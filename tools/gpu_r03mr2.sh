#!/bin/bash
set -e
OUT=${1:-gpurun_out/r03mr2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_bench.py > "$OUT/tests.log" 2>&1
