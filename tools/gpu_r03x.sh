#!/bin/bash
# option sweep on the Hilbert-ordered mesh: XCD run length, entities per wave
set -e
OUT=${1:-gpurun_out/r03x}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 tools/abstep.py --rounds 6 --steps 5 --variants xcd=64 xcd=32 xcd=128 xcd=256 xcd=1 epw=1 epw=4 > "$OUT/ab.json"
