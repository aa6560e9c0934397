#!/bin/bash
# transport slot order within XCD runs (option trorder = R): parity, then interleaved A/B
set -e
OUT=${1:-gpurun_out/r03t2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_transport.py > "$OUT/tests.log" 2>&1
timeout -k 10 400 python3 tools/kbench.py --transport --rounds 4 --variants trorder=0 trorder=1 trorder=64 trorder=256 trorder=1024 trorder=4096 > "$OUT/kb.json"
