#!/bin/bash
# option fusecopy: parity, then whole-step A/B and per-task times
set -e
OUT=${1:-gpurun_out/r03n}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fusedamp or main_rg or setup" tests/test_gpu_bench.py > "$OUT/tests.log" 2>&1
timeout -k 10 300 python3 tools/abstep.py --variants "fusecopy=1" "fusecopy=0" > "$OUT/ab_big.json"
timeout -k 10 200 python3 tools/abstep.py --ncells 2562 --steps 20 --variants "fusecopy=1" "fusecopy=0" > "$OUT/ab_small.json"
timeout -k 10 300 python3 tools/kbench.py --rounds 3 --variants "fusecopy=1" "fusecopy=0" > "$OUT/kb.json"
