#!/bin/bash
# whole-step A/B of the round-3 fusion options (each variant from the defaults)
set -e
OUT=${1:-gpurun_out/r03l}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=("hfuse=1" "hfuse=0" "hfuse=0,tmedge=0" "hfuse=0,fusesml=0" "hfuse=0,tmedge=0,fusesml=0" "hfuse=0,tmedge=0,fusesml=0,fusedamp=0,fusesetup=0")
timeout -k 10 400 python3 tools/abstep.py --variants "${V[@]}" > "$OUT/ab_big.json"
timeout -k 10 200 python3 tools/abstep.py --ncells 2562 --steps 20 --variants "${V[@]}" > "$OUT/ab_small.json"
timeout -k 10 300 python3 tools/kbench.py --rounds 3 --variants "hfuse=1" "hfuse=0,tmedge=0,fusesml=0" > "$OUT/kb.json"
