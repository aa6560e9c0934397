#!/usr/bin/env python3
"""One rank of an N-way decomposition on one GPU: rank R's subdomain of the benchmark mesh
with its whole launch sequence -- interior / boundary launches, halo packs and unpacks --
and the stub transport in place of RCCL (mpas_halo_stub: a device copy stands in for the
wire), so everything but the wire time is timed.  The per-rank critical path of the
8-GPU run (<= 2.1 ms/step at x1.163842 / 8 for 6x on 8 GPUs).

    python tools/rank_sim.py [--parts 8] [--rank 0] [--ncells 163842] [--steps 20]
                             [--graph 0|1] [--overlap 0|1] [--physics 0|1|2] [--transport 0|1]
                             [--latency-us US]

Prints one JSON line: per-rank ms/step (median of per-step HIP events), the host enqueue
time per step, exchanges per step, and the undecomposed step for comparison."""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mpas-regent_amd")]
import bench  # noqa: E402
from mpasdyn import decomp, lib  # noqa: E402
from mpasdyn import tasks as T  # noqa: E402


def timed(ctx, dt, steps, warm=3):
    hip = bench.Hip()
    for _ in range(warm):
        T.atm_srk3(ctx, dt, 1)
    ctx.sync()
    evs = [hip.event() for _ in range(steps + 1)]
    stream = ctx.stream()
    host = []
    hip.record(evs[0], stream)
    for i in range(steps):
        a = time.perf_counter()
        T.atm_srk3(ctx, dt, 1)
        host.append(time.perf_counter() - a)
        hip.record(evs[i + 1], stream)
    ctx.sync()
    ms = [hip.elapsed_ms(evs[i], evs[i + 1]) for i in range(steps)]
    return statistics.median(ms), 1e3 * statistics.median(host)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--ncells", type=int, default=163842)
    ap.add_argument("--levels", type=int, default=56)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--overlap", type=int, default=1)
    ap.add_argument("--full", type=int, default=1, help="also time the undecomposed mesh")
    ap.add_argument("--option", action="append", default=[])
    ap.add_argument("--physics", type=int, default=0, choices=[0, 1, 2])
    ap.add_argument("--transport", type=int, default=0)
    ap.add_argument("--latency-us", type=int, default=0,
                    help="the stub's modelled wire latency per exchange (a device-side wait on the halo stream)")
    ap.add_argument("--debug", type=int, default=0)
    a = ap.parse_args()
    if a.transport and not a.physics:
        a.physics = 1
    m, st = bench.build_inputs(a.ncells, a.levels, zero_based=bool(a.physics))
    dt = bench.dt_for(a.ncells)
    out = {"workload": f"x1.{a.ncells} x {a.levels}, rank {a.rank} of {a.parts}, stub transport"
                       + (f", physics {a.physics}" if a.physics else "") + (", transport" if a.transport else ""),
           "graph_halo": a.graph, "overlap": a.overlap, "latency_us_per_exchange": a.latency_us}

    def opts(ctx):
        ctx.set_option("physics", a.physics)
        ctx.set_option("transport", a.transport)
    if a.full:
        ctx = lib.Context(m.nCells, m.nEdges, m.nVertices, a.levels)
        opts(ctx)
        bench.upload_inputs(ctx, st)
        out["full_ms_per_step"], _ = timed(ctx, dt, a.steps)
        ctx.close()
    dec = decomp.Decomposition(st, a.parts)
    lst = dec.local_state(a.rank)
    dims = (*dec.n_local(a.rank), a.levels)
    ctx = lib.Context(*dims)
    lib.setup_subdomain(ctx, dec, a.rank)
    lib.halo_stub(ctx)
    opts(ctx)
    ctx.set_option("overlap", a.overlap)
    ctx.set_option("graph_halo", a.graph)
    if a.latency_us:
        ctx.set_option("stub_latency_us", a.latency_us)
    for kv in a.option:
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    bench.upload_inputs(ctx, lst)
    ex0, _ = lib.halo_stats(ctx)
    out["rank_ms_per_step"], out["rank_host_enqueue_ms"] = timed(ctx, dt, a.steps)
    ex1, _ = lib.halo_stats(ctx)
    out["exchanges_per_step"] = round((ex1 - ex0) / (a.steps + 3), 2)
    out["graph_captures"] = ctx.get_option("graph_captures")
    out["graph_launches"] = ctx.get_option("graph_launches")
    out["graph_fallbacks"] = ctx.get_option("graph_fallbacks")
    if a.debug:  # the halo bookkeeping at each step's start
        hs = []
        for _ in range(6):
            hs.append(ctx.get_option("halo_state") % 100000)
            T.atm_srk3(ctx, dt, 1)
        out["halo_states"] = hs
    out["owned"] = list(dec.n_owned(a.rank))
    out["interior"] = list(dec.n_interior(a.rank))
    out["local"] = list(dims[:3])
    if a.full:
        out[f"speedup_bound_{a.parts}"] = round(out["full_ms_per_step"] / out["rank_ms_per_step"], 3)
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
