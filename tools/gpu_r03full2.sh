#!/bin/bash
# the whole GPU suite (as the driver runs it), then smoke
set -e
OUT=${1:-gpurun_out/r03full2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
