#!/bin/bash
# transport pair-layout iteration: parity of every test that touches the x8 fields, then
# interleaved whole-step A/B (bench --transport workload) of the HEAD build (abl/base) and
# the timing variants in abl/ against the in-tree build
set -e
OUT=${1:-gpurun_out/r03t}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_transport.py tests/test_gpu_views.py tests/test_gpu_bounds.py tests/test_gpu_graph.py > "$OUT/tests.log" 2>&1
for r in 1 2; do
  timeout -k 10 200 python3 tools/kbench.py --transport --rounds 3 --variants xcd=64 > "$OUT/new_$r.json"
  for so in abl/*.so; do
    timeout -k 10 200 env MPAS_LIB=$so python3 tools/kbench.py --transport --rounds 3 --variants xcd=64 > "$OUT/$(basename $so .so)_$r.json"
  done
done
