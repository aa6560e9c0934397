#!/bin/bash
# per-kernel HBM traffic and L2 hit rates of the headline step (Hilbert mesh)
set -e
OUT=${1:-gpurun_out/r03pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 bash tools/tr_kernels.sh "$OUT/k" --option xcd=64
