#!/bin/bash
# dyn_tend C vertex width (option cve): full GPU suite, interleaved step A/B of the widths
# at x1.2562 and x1.163842, then the headline bench line and its rocprofv3 trace
set -e
OUT=${1:-gpurun_out/r03v8}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 200 python3 tools/abstep.py --ncells 2562 --rounds 6 --steps 20 --variants cve=0 cve=1 cve=4 cve=8 > "$OUT/ab_cve_x1.2562.json"
timeout -k 10 300 python3 tools/abstep.py --ncells 163842 --rounds 4 --steps 5 --variants cve=0 cve=1 cve=4 cve=8 > "$OUT/ab_cve_x1.163842.json"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --traffic off > "$OUT/trace.log" 2>&1
