#!/bin/bash
# Per-kernel time and HBM bytes of the transport kernels (k_tr_*) and the rest of the
# transport step: kernel trace, then FETCH_SIZE, WRITE_SIZE and TCC hit/miss passes (one
# counter group per run).  usage: bash tools/tr_kernels.sh OUTDIR [bench args...]
set -e
OUT=${1:-gpurun_out/trk}
shift || true
ARGS=${@:---transport}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py $ARGS --steps 1 --warmup 0 --no-cpu-baseline --traffic off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv -- python3 $B > "$OUT/trace.log" 2>&1
for P in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $P -d "$OUT/pmc_$n" -o pmc --output-format csv -- python3 $B > "$OUT/pmc_$n.log" 2>&1
done
python3 tools/pmc_kernels.py "$OUT"/pmc_* --match "k_" > "$OUT/kernels.txt"
