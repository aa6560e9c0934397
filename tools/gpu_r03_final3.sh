#!/bin/bash
# the headline bench line and the rocprofv3 kernel trace + stats of the same command, one box
set -e
OUT=${1:-gpurun_out/r03v7}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --traffic off > "$OUT/trace.log" 2>&1
