#!/usr/bin/env python3
"""Whole-step A/B in one process: the benchmark workload built once, interleaved rounds of
K atm_srk3 steps (HIP graph replay, as bench.py times them) under each option set (options a variant does not name at their defaults); per
variant the median per-step device time over all rounds (HIP events between steps).

usage: python tools/abstep.py [--ncells 163842] [--rounds 6] [--steps 5] [--physics N] [--transport]
       --variants "fusesetup=1" "fusesetup=0"
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
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--physics", type=int, default=0, choices=[0, 1, 2])
    ap.add_argument("--transport", action="store_true", help="physics 1 + the scalar transport (bench --transport)")
    a = ap.parse_args()
    physics = max(a.physics, 1 if a.transport else 0)
    m, st = bench.build_inputs(a.ncells, a.levels, zero_based=physics)
    ctx = lib.Context(m.nCells, m.nEdges, m.nVertices, a.levels)
    ctx.set_option("physics", physics)
    ctx.set_option("transport", int(a.transport))
    bench.upload_inputs(ctx, st)
    dt = bench.dt_for(a.ncells)
    hip = bench.Hip()
    stream = ctx.stream()
    evs = [hip.event() for _ in range(a.steps + 1)]
    res = {v: [] for v in a.variants}
    # every option a variant names starts from its default in every variant (a variant
    # lists only what it changes)
    keys = {kv.split("=")[0] for v in a.variants for kv in v.split(",")}
    base = {k: ctx.get_option(k) for k in keys}
    for _ in range(a.rounds):
        for v in a.variants:
            for k, val in base.items():
                ctx.set_option(k, val)
            for kv in v.split(","):
                k, val = kv.split("=")
                ctx.set_option(k, int(val))
            T.atm_srk3(ctx, dt, 1)  # (re-capture after the option change)
            T.atm_srk3(ctx, dt, 1)
            ctx.sync()
            hip.record(evs[0], stream)
            for i in range(a.steps):
                T.atm_srk3(ctx, dt, 1)
                hip.record(evs[i + 1], stream)
            ctx.sync()
            res[v] += [hip.elapsed_ms(evs[i], evs[i + 1]) for i in range(a.steps)]
    out = {v: {"median_ms": round(statistics.median(x), 4), "min_ms": round(min(x), 4), "n": len(x)}
           for v, x in res.items()}
    out["workload"] = f"x1.{a.ncells} x {a.levels}, physics {physics}, transport {int(a.transport)}"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
