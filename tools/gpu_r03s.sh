#!/bin/bash
set -e
OUT=${1:-gpurun_out/r03s}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/abstep.py --rounds 6 --variants "hfuse=2" "hfuse=1" > "$OUT/ab_big.json"
timeout -k 10 300 python3 tools/kbench.py --rounds 3 --variants "hfuse=2" "hfuse=1" > "$OUT/kb.json"
