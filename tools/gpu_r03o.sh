#!/bin/bash
# transport edge groups (option tredge): parity, A/B at x1.163842 x 56 x 8; dyn_tend gather cost
set -e
OUT=${1:-gpurun_out/r03o}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_transport.py > "$OUT/tests.log" 2>&1
timeout -k 10 400 python3 tools/kbench.py --rounds 3 --transport --variants "tredge=1" "tredge=0" > "$OUT/kb_tr.json"
bash tools/gather_cost.sh run "$OUT/gcost"
