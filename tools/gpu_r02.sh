#!/bin/bash
# Round-2 GPU evidence (run on the GPU box from the repo root): bench lines (headline with
# live traffic + cpu_baseline, MPAS dynamics, transport, small meshes with and without the
# HIP graph), the rocprofv3 kernel trace + stats of the headline bench.
# usage: bash tools/gpu_r02.sh OUT
set -e
OUT=${1:-gpurun_out/r02}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 python3 bench.py --physics 2 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_physics2.json" 2>> "$OUT/bench.err"
timeout -k 10 300 python3 bench.py --transport --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_transport.json" 2>> "$OUT/bench.err"
for n in 2562 40962; do
  timeout -k 10 200 python3 bench.py --ncells $n --steps 50 --warmup 5 --no-cpu-baseline --traffic off > "$OUT/bench_x1.${n}_graph.json" 2>> "$OUT/bench.err"
  timeout -k 10 200 python3 bench.py --ncells $n --steps 50 --warmup 5 --no-cpu-baseline --traffic off --option graph=0 > "$OUT/bench_x1.${n}_nograph.json" 2>> "$OUT/bench.err"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --traffic off > "$OUT/trace.log" 2>&1
