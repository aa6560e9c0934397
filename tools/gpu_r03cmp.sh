#!/bin/bash
# bench.py against tools/abstep.py on one box
set -e
OUT=${1:-gpurun_out/r03cmp}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu-baseline --traffic off > "$OUT/b1.json" 2> "$OUT/err"
timeout -k 10 300 python3 tools/abstep.py --rounds 4 --steps 5 --variants xcd=64 > "$OUT/ab.json"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --traffic off --steps 20 > "$OUT/b2.json" 2>> "$OUT/err"
timeout -k 10 300 python3 bench.py > "$OUT/b3.json" 2>> "$OUT/err"
