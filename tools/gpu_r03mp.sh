#!/bin/bash
# the multi-process socket-transport test
set -e
OUT=${1:-gpurun_out/r03mp}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multiproc.py > "$OUT/tests.log" 2>&1
