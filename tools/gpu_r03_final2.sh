#!/bin/bash
# Round-3 final bench lines (Hilbert-numbered meshes): headline with traffic and cpu
# baseline, its kernel trace, transport, MPAS dynamics, small meshes, config-5 mesh
set -e
OUT=${1:-gpurun_out/r03v6}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --traffic off > "$OUT/trace.log" 2>&1
timeout -k 10 400 python3 bench.py --transport --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_transport.json" 2>> "$OUT/bench.err"
timeout -k 10 400 python3 bench.py --physics 2 --steps 10 --warmup 3 --no-cpu-baseline --traffic off > "$OUT/bench_physics2.json" 2>> "$OUT/bench.err"
for n in 2562 40962; do
  timeout -k 10 200 python3 bench.py --ncells $n --steps 50 --warmup 5 --no-cpu-baseline --traffic off > "$OUT/bench_x1.${n}.json" 2>> "$OUT/bench.err"
done
timeout -k 10 600 python3 bench.py --ncells 655362 --steps 5 --warmup 2 --no-cpu-baseline --traffic off > "$OUT/bench_x1.655362.json" 2>> "$OUT/bench.err"
timeout -k 10 600 python3 bench.py --ncells 655362 --transport --steps 5 --warmup 2 --no-cpu-baseline --traffic off > "$OUT/bench_x1.655362_transport.json" 2>> "$OUT/bench.err"
