#!/usr/bin/env python3
"""Per-task A/B timing in one process (cdna guide §5.4 rule 24): builds the benchmark
workload once and runs interleaved rounds of full RK3 steps under each option set,
reporting the median per-task device time (HIP events on the task stream).

usage: python tools/kbench.py [--ncells 163842] [--levels 56] [--rounds 5] [--physics N] [--transport]
       --variants "xcd=1" "xcd=0"
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mpas-regent_amd")]

import bench  # noqa: E402
from mpasdyn import lib  # noqa: E402
from mpasdyn import tasks as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ncells", type=int, default=163842)
    ap.add_argument("--levels", type=int, default=56)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", nargs="+", default=["xcd=1", "xcd=0"])
    ap.add_argument("--physics", type=int, default=0)
    ap.add_argument("--transport", action="store_true", help="physics 1 + the scalar transport (bench --transport)")
    a = ap.parse_args()
    physics = max(a.physics, 1 if a.transport else 0)
    m, st = bench.build_inputs(a.ncells, a.levels, zero_based=physics)
    ctx = lib.Context(m.nCells, m.nEdges, m.nVertices, a.levels)
    ctx.set_option("physics", physics)
    ctx.set_option("transport", int(a.transport))
    bench.upload_inputs(ctx, st)
    dt = bench.dt_for(a.ncells)
    T.atm_srk3(ctx, dt, 1)
    res = {v: {} for v in a.variants}
    keys = {kv.split("=")[0] for v in a.variants for kv in v.split(",")}
    base = {k: ctx.get_option(k) for k in keys}  # (a variant lists only what it changes)
    for r in range(a.rounds):
        for v in a.variants:
            for k, val in base.items():
                ctx.set_option(k, val)
            for kv in v.split(","):
                k, val = kv.split("=")
                ctx.set_option(k, int(val))
            T.atm_srk3(ctx, dt, 1)  # untimed: one-time work an option change triggers (tile builds)
            ctx.timing(True)
            ctx.timing_reset()
            T.atm_srk3(ctx, dt, 1)
            ctx.sync()
            for name, (calls, ms) in ctx.timing_report().items():
                res[v].setdefault(name, []).append(ms)
            ctx.timing(False)
    out = {}
    for v in a.variants:
        out[v] = {n: round(statistics.median(x), 4) for n, x in res[v].items()}
        out[v]["step_ms"] = round(sum(out[v].values()), 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
