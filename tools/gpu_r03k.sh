#!/bin/bash
set -e
OUT=${1:-gpurun_out/r03k}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_main_run.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_bench.py} > "$OUT/tests.log" 2>&1
timeout -k 10 300 python3 tools/abstep.py --variants "hfuse=1" "hfuse=0" "hfuse=0,tmedge=0,fusesml=0" "hfuse=0,tmedge=0,fusesml=0,fusedamp=0,fusesetup=0" > "$OUT/ab_big.json"
timeout -k 10 200 python3 tools/abstep.py --ncells 2562 --steps 20 --variants "hfuse=1" "hfuse=0" "hfuse=0,tmedge=0,fusesml=0" "hfuse=0,tmedge=0,fusesml=0,fusedamp=0,fusesetup=0" > "$OUT/ab_small.json"
timeout -k 10 300 python3 tools/kbench.py --rounds 3 --variants "hfuse=1" "hfuse=0,tmedge=0,fusesml=0,fusedamp=0,fusesetup=0" > "$OUT/kb.json"
