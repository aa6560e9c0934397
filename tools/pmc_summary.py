#!/usr/bin/env python3
"""Summarise rocprofv3 output for the benchmark: per-kernel average duration from the
kernel trace and per-dispatch HBM bytes from separate FETCH_SIZE / WRITE_SIZE passes.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128-B read
request, i.e. half the bytes of a coalesced stream, so fetched bytes = 2 * FETCH_SIZE KB
* 1024.  The factor is re-derived here from k_setup_cells / k_setup_edges, whose bytes
are known exactly (pure copies of L levels of each column), and the measured factor is
what is applied and reported.

usage: pmc_summary.py --trace DIR --fetch DIR --write DIR --dims nC nE nV L --out FILE
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def read_counter(d, name):
    rows = list(csv.DictReader(open(glob.glob(os.path.join(d, "*counter_collection.csv"))[0])))
    acc = defaultdict(list)
    for r in rows:
        if r["Counter_Name"] == name:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--dims", nargs=4, type=int)
    ap.add_argument("--out")
    a = ap.parse_args()
    nC, nE, nV, L = a.dims
    out = {"dims": a.dims, "kernels": {}}
    if a.trace:
        for r in csv.DictReader(open(glob.glob(os.path.join(a.trace, "*kernel_stats.csv"))[0])):
            out["kernels"].setdefault(r["Name"], {})["avg_us"] = float(r["AverageNs"]) / 1e3
            out["kernels"][r["Name"]]["calls"] = int(r["Calls"])
    fetch, _ = read_counter(a.fetch, "FETCH_SIZE") if a.fetch else ({}, {})
    write, _ = read_counter(a.write, "WRITE_SIZE") if a.write else ({}, {})
    # calibration: setup copies read 6 C3 + (cells) / 2 E3 (edges) arrays of L levels
    known = {"k_setup_cells": 6 * 8 * nC * L, "k_setup_edges": 2 * 8 * nE * L}
    kn = [k for k in known if any(k in n for n in fetch)]
    factor = None
    if kn:
        ratios = []
        for k in kn:
            name = next(n for n in fetch if k in n)
            ratios.append(known[k] / (fetch[name] * 1024.0))
        factor = sum(ratios) / len(ratios)
    out["fetch_factor_measured"] = factor
    f = factor if factor else 2.0
    for name in set(fetch) | set(write):
        short = name.split("(")[0].split("<")[0].split("::")[-1]
        d = out["kernels"].setdefault(short, {})
        d["fetch_bytes"] = fetch.get(name, 0.0) * 1024.0 * f
        d["write_bytes"] = write.get(name, 0.0) * 1024.0
        d["hbm_bytes"] = d["fetch_bytes"] + d["write_bytes"]
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1, sort_keys=True)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1].get("avg_us", 0) * kv[1].get("calls", 0)):
        print(f"{k:34s} avg_us={v.get('avg_us', 0):9.1f} calls={v.get('calls', 0):4d} "
              f"fetch_MB={v.get('fetch_bytes', 0) / 1e6:9.1f} write_MB={v.get('write_bytes', 0) / 1e6:8.1f} "
              f"GB/s={(v.get('hbm_bytes', 0) / (v.get('avg_us', 1e9) * 1e-6) / 1e9) if v.get('avg_us') else 0:8.1f}")
    print("fetch factor", factor)


if __name__ == "__main__":
    main()
