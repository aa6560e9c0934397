#!/bin/bash
# per-kernel time and HBM bytes of the transport kernels, trorder 0 and 64
set -e
OUT=${1:-gpurun_out/r03t4}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 bash tools/tr_kernels.sh "$OUT/o0" --transport
timeout -k 10 400 bash tools/tr_kernels.sh "$OUT/o64" --transport --option trorder=64
