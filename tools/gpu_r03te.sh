#!/bin/bash
# transport edge kernel slot order (option trorder_e)
set -e
OUT=${1:-gpurun_out/r03te}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_transport.py > "$OUT/tests.log" 2>&1
timeout -k 10 500 python3 tools/kbench.py --transport --rounds 4 --variants trorder_e=0 trorder_e=16 trorder_e=32 trorder_e=128 trorder_e=256 trorder_e=512 trorder_e=1 > "$OUT/kb.json"
