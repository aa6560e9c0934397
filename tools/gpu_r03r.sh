#!/bin/bash
# round-3 evidence: the default bench line (cpu baseline + live traffic), its kernel trace,
# the other single-GPU configs, the transport and MPAS-dynamics workloads
set -e
OUT=${1:-gpurun_out/r03r}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --traffic off > "$OUT/trace.json" 2> "$OUT/trace.err"
for n in 2562 40962; do
  timeout -k 10 200 python3 bench.py --ncells $n --steps 50 --warmup 5 --no-cpu-baseline --traffic off > "$OUT/bench_x1.$n.json" 2>> "$OUT/bench.err"
done
timeout -k 10 300 python3 bench.py --transport --steps 10 --warmup 3 --no-cpu-baseline --traffic off > "$OUT/bench_transport.json" 2>> "$OUT/bench.err"
timeout -k 10 300 python3 bench.py --physics 2 --steps 10 --warmup 3 --no-cpu-baseline --traffic off > "$OUT/bench_physics2.json" 2>> "$OUT/bench.err"
