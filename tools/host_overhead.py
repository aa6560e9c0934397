#!/usr/bin/env python3
"""Host enqueue time of one RK3 step (the C-ABI call returns once every kernel is queued)
against its device time: whether the host keeps ahead of the GPU, at full size and at
1/8 of the mesh (the local mesh of rank 0 of an 8-GPU decomposition, without the halo
exchanges, which add a pack, an RCCL group and an unpack per exchange).

usage (GPU box): python tools/host_overhead.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mpas-regent_amd")]
import bench  # noqa: E402
from mpasdyn import decomp, lib  # noqa: E402
from mpasdyn import tasks as T  # noqa: E402


def run(ctx, dt, n=10):
    T.atm_srk3(ctx, dt, 1)
    ctx.sync()
    host = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        T.atm_srk3(ctx, dt, 1)
        host.append(time.perf_counter() - a)
    ctx.sync()
    wall = (time.perf_counter() - t0) / n
    return 1e3 * sorted(host)[n // 2], 1e3 * wall


def main():
    m, st = bench.build_inputs(163842, 56)
    dt = bench.dt_for(163842)
    ctx = lib.Context(m.nCells, m.nEdges, m.nVertices, 56)
    bench.upload_inputs(ctx, st)
    h, w = run(ctx, dt)
    print(f"full mesh: host enqueue {h:.3f} ms/step, wall {w:.3f} ms/step")
    ctx.close()
    dec = decomp.Decomposition(st, 8)
    lst = dec.local_state(0)
    dims = (*dec.n_local(0), 56)
    ctx = lib.Context(*dims)  # the subdomain's local mesh alone (no halo: kernel launches only)
    bench.upload_inputs(ctx, lst)
    h, w = run(ctx, dt)
    print(f"1/8 subdomain without its halo: host enqueue {h:.3f} ms/step, wall {w:.3f} ms/step")
    ctx.close()


if __name__ == "__main__":
    main()
