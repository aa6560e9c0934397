#!/bin/bash
# transport option trepw (two edges per wavefront): parity, then interleaved A/B
set -e
OUT=${1:-gpurun_out/r03t6}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_transport.py > "$OUT/tests.log" 2>&1
for r in 1 2; do
  timeout -k 10 300 python3 tools/kbench.py --transport --rounds 3 --variants trepw=1 trepw=2 trepw=2,trorder=256 trepw=2,trorder=0 > "$OUT/new_$r.json"
done
