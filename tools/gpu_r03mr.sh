#!/bin/bash
# the multi-rank flow of bench.py (spawned ranks, TCP rendezvous, decomposition, max-over-
# ranks timing, one JSON line) rehearsed on one GPU with the socket halo transport
set -e
OUT=${1:-gpurun_out/r03mr}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 2 --halo socket --steps 3 --warmup 1 --no-cpu-baseline --traffic off > "$OUT/bench_g2_socket.json" 2> "$OUT/g2.err"
timeout -k 10 400 python3 bench.py --gpus 4 --halo socket --ncells 40962 --steps 3 --warmup 1 --no-cpu-baseline --traffic off > "$OUT/bench_g4_socket_x1.40962.json" 2> "$OUT/g4.err"
timeout -k 10 400 python3 bench.py --gpus 1 --decompose --steps 5 --warmup 2 --no-cpu-baseline --traffic off > "$OUT/bench_g1_decompose.json" 2> "$OUT/g1.err"
