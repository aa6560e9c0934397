#!/bin/bash
# Interleaved whole-step A/B of library builds (run on the GPU box from the repo root):
# kbench.py under MPAS_LIB=<each .so> (the in-tree build for "new"), two rounds.
# usage: bash tools/kbench_ab.sh OUTDIR LIB1.so [LIB2.so ...]
set -e
OUT=$1; shift
mkdir -p "$OUT"
for r in 1 2; do
  timeout -k 10 120 python3 tools/kbench.py --rounds 3 --variants xcd=64 > "$OUT/new_$r.json" 2>/dev/null
  for so in "$@"; do
    timeout -k 10 120 env MPAS_LIB=$so python3 tools/kbench.py --rounds 3 --variants xcd=64 > "$OUT/$(basename $so .so)_$r.json" 2>/dev/null
  done
done
python3 - "$OUT" <<'PY'
import glob, json, os, sys
out = sys.argv[1]
res = {}
for f in sorted(glob.glob(f"{out}/*_[12].json")):
    name = os.path.basename(f).rsplit("_", 1)[0]
    d = list(json.load(open(f)).values())[0]
    for k, v in d.items():
        res.setdefault(name, {}).setdefault(k, []).append(v)
names = sorted(res)
keys = list(res[names[0]])
with open(f"{out}/ab.txt", "w") as fh:
    fh.write("%-42s" % "task" + "".join("%12s" % n for n in names) + "\n")
    for k in keys:
        fh.write("%-42s" % k[:42] + "".join("%12.4f" % (sum(res[n][k]) / len(res[n][k])) for n in names) + "\n")
PY
cat "$OUT/ab.txt"
