#!/bin/bash
# final build of round 3: full GPU suite, smoke(), the headline bench line and its rocprofv3 trace
set -e
OUT=${1:-gpurun_out/r03v9}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --traffic off > "$OUT/trace.log" 2>&1
