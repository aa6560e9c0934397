#!/bin/bash
# kernel traces (timestamps) of the small and the headline step with the new defaults
set -e
OUT=${1:-gpurun_out/r03m}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/small" -o kt --output-format csv -- python3 bench.py --ncells 2562 --steps 20 --warmup 5 --no-cpu-baseline --traffic off > "$OUT/small.json" 2> "$OUT/small.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/big" -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --traffic off > "$OUT/big.json" 2> "$OUT/big.err"
timeout -k 10 200 python3 bench.py --ncells 2562 --steps 50 --warmup 5 --no-cpu-baseline --traffic off > "$OUT/bench_x1.2562.json"
