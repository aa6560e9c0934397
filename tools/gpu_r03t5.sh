#!/bin/bash
# transport option trsu: parity, then interleaved A/B (in-tree and the MINW=4 build)
set -e
OUT=${1:-gpurun_out/r03t5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_transport.py > "$OUT/tests.log" 2>&1
for r in 1 2; do
  timeout -k 10 300 python3 tools/kbench.py --transport --rounds 3 --variants trorder=64,trsu=0 trorder=64,trsu=1 trorder=16,trsu=0 > "$OUT/new_$r.json"
  timeout -k 10 300 env MPAS_LIB=abl/libmpasdyn_tru4.so python3 tools/kbench.py --transport --rounds 3 --variants trorder=64,trsu=1 > "$OUT/tru4_$r.json"
done
