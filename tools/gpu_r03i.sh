#!/bin/bash
set -e
OUT=${1:-gpurun_out/r03i}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "solve or srk3 or fusedamp" > "$OUT/tests.log" 2>&1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_mpas_dynamics.py tests/test_gpu_decomp.py > "$OUT/tests2.log" 2>&1
timeout -k 10 300 python3 tools/abstep.py --variants "epw=2" "epw=1" "epw=4" > "$OUT/ab_epw.json"
timeout -k 10 300 python3 tools/kbench.py --rounds 4 --variants "epw=2" "epw=1" "epw=4" > "$OUT/kb_epw.json"
