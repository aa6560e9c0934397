#!/bin/bash
# Profile of bench.py --transport (the MPAS solver + the monotonic scalar transport) on
# the GPU box from the repo root: kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes
# (separate, no trace domains), the per-task summary, and one full bench line.
# usage: bash tools/profile_transport.sh OUTDIR
set -e
OUT=${1:-gpurun_out/prof_tr}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --transport --steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv -- python3 $B > "$OUT/trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o pmc --output-format csv -- python3 bench.py --transport --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o pmc --output-format csv -- python3 bench.py --transport --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/write.log" 2>&1
python3 tools/pmc_summary.py --physics --trace "$OUT/trace" --fetch "$OUT/fetch" --write "$OUT/write" \
    --dims 163842 491520 327680 56 --out "$OUT/pmc_transport_x1.163842_L56.json" > "$OUT/pmc_summary.txt"
timeout -k 10 600 python3 bench.py --transport > "$OUT/bench_transport.json" 2> "$OUT/bench.err"
