#!/bin/bash
# Per-kernel A/B of two library builds under rocprofv3 --kernel-trace --stats (run on
# the GPU box from the repo root): bench.py steps with the default build and with
# MPAS_LIB=$2, then a side-by-side of the average kernel durations.
# usage: bash tools/ktrace_ab.sh OUTDIR OLD_SO
set -e
OUT=${1:-gpurun_out/kab}
OLD=$2
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 1 --no-cpu-baseline"
# interleaved new, old, old, new (the first run on a box tends to be the slowest)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/new" -o kt --output-format csv -- python3 $B > "$OUT/new.log" 2>&1
MPAS_LIB=$OLD timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/old" -o kt --output-format csv -- python3 $B > "$OUT/old.log" 2>&1
MPAS_LIB=$OLD timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/old2" -o kt --output-format csv -- python3 $B > "$OUT/old2.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/new2" -o kt --output-format csv -- python3 $B > "$OUT/new2.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys
out = sys.argv[1]
def load1(d):
    f = glob.glob(f"{out}/{d}/**/kt_kernel_stats.csv", recursive=True)[0]
    return {r["Name"]: (int(r["Calls"]), float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(f))}
def load(a, b):
    x, y = load1(a), load1(b)
    return {k: (x[k][0], 0.5 * (x[k][1] + y.get(k, x[k])[1])) for k in x}
o, n = load("old", "old2"), load("new", "new2")
rows = sorted(n, key=lambda k: -n[k][0] * n[k][1])
with open(f"{out}/ab.txt", "w") as fh:
    for k in rows[:30]:
        oc = o.get(k, (0, float("nan")))
        fh.write(f"{k[:70]:70s} {n[k][0]:5d} new {n[k][1]:9.1f} us  old {oc[1]:9.1f} us  {100*(n[k][1]/oc[1]-1):+6.1f}%\n")
PY
cat "$OUT/ab.txt"
