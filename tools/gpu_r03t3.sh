#!/bin/bash
# transport: scratch at pitch L with range-checked buffer access; parity then A/B
set -e
OUT=${1:-gpurun_out/r03t3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_transport.py tests/test_gpu_bounds.py tests/test_gpu_views.py > "$OUT/tests.log" 2>&1
for r in 1 2; do
  timeout -k 10 300 python3 tools/kbench.py --transport --rounds 3 --variants trorder=0 trorder=64 > "$OUT/new_$r.json"
  timeout -k 10 300 env MPAS_LIB=abl/libmpasdyn_base.so python3 tools/kbench.py --transport --rounds 3 --variants trorder=0 > "$OUT/base_$r.json"
done
