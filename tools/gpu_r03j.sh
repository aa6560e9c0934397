#!/bin/bash
set -e
OUT=${1:-gpurun_out/r03j}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_main_run.py tests/test_gpu_configs.py > "$OUT/tests.log" 2>&1
timeout -k 10 300 python3 tools/abstep.py --variants "tmedge=1,fusesml=1" "tmedge=0,fusesml=1" "tmedge=1,fusesml=0" "tmedge=0,fusesml=0" > "$OUT/ab_tme.json"
timeout -k 10 300 python3 tools/kbench.py --rounds 3 --variants "tmedge=1,fusesml=1" "tmedge=0,fusesml=0" > "$OUT/kb_tme.json"
timeout -k 10 200 python3 tools/abstep.py --ncells 2562 --steps 20 --variants "tmedge=1,fusesml=1" "tmedge=0,fusesml=0" > "$OUT/ab_small.json"
