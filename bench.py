#!/usr/bin/env python3
"""Benchmark of the RK3 dynamics hot path (atm_srk3, rk_timestep.rg:361-500) on MI355X.

Metric (BASELINE.json): Mcell-columns/s per RK3 step at x1.163842 x 56 levels, plus the
achieved HBM bandwidth of the dominant kernel against the 8 TB/s roofline.

One step = one atm_srk3 call: setup, moist, 2x vert_imp, 3x dyn_tend (rk_step 0,1,2 --
the MPAS schedule of SURVEY §8.5), 3x smlstep, 7x acoustic + 7x divergence damping,
3x solve_diagnostics, substep_finish (28 tasks).  Inputs are resident in HBM before the
timed region: the x1.163842 icosahedral mesh (mpasdyn.mesh) with its one-time
precompute uploaded from the host, and the 3-D state filled on the device by the
seeded generator (data: synthetic, seed 20211015).

    python bench.py [--gpus N --steps K --warmup W]
N > 1 runs under torch.distributed.run, one process per GPU: the same x1.163842 mesh is
split into N subdomains (mpasdyn/decomp.py: contiguous blocks of the Morton-ordered
cells, edges/vertices with their first cell/edge, ghosts = everything an owned entity
reaches through an index array), and the ranks exchange halos with RCCL send/recv
before every kernel that gathers a field another rank wrote (csrc/mpas_halo.h).  Total
work is fixed ("scaling": "strong"); `value` = global cell columns / step time.
`--replicas` instead runs a full-mesh replica per rank (weak scaling, no collective).
Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mpas-regent_amd"))

import numpy as np  # noqa: E402

METRIC = "Mcell-columns/sec per RK3 step; achieved HBM GB/s; x1.163842×56L"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak
LEVEL_OF = {2562: 4, 10242: 5, 40962: 6, 163842: 7, 655362: 8}
SEED = 20211015


class Hip:
    """the few HIP runtime calls the timing needs (events on the library's stream)"""

    def __init__(self):
        self.h = ctypes.CDLL("libamdhip64.so")
        self.h.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self.h.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        self.h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]

    def event(self):
        e = ctypes.c_void_p()
        assert self.h.hipEventCreate(ctypes.byref(e)) == 0
        return e

    def record(self, e, stream):
        assert self.h.hipEventRecord(e, ctypes.c_void_p(stream)) == 0

    def elapsed_ms(self, e0, e1):
        assert self.h.hipEventSynchronize(e1) == 0
        ms = ctypes.c_float()
        assert self.h.hipEventElapsedTime(ctypes.byref(ms), e0, e1) == 0
        return float(ms.value)


def build_inputs(ncells, L, zero_based=False):
    """the mesh and its one-time precompute (host); the 3-D state is filled on the device.
    zero_based: mpas-mode (0-based) connectivity, the ids the MPAS solver and the transport
    are defined on (the default keeps the reference's raw 1-based ids, Q1)"""
    from mpasdyn import build_state as bs
    from mpasdyn import mesh
    m = mesh.icosahedral(LEVEL_OF[ncells])
    if zero_based:
        m = mesh.zero_based(m)
    st = bs.build_state(m, L, "physical", mesh_only=True)
    return m, st


def dt_for(ncells):
    # dt = 720 * 2**(4-k) s for x1.(10*4**k+2)
    return 720.0 * 2.0 ** (4 - LEVEL_OF[ncells])


def upload_inputs(ctx, st):
    from mpasdyn.registry import FIELDS
    ctx.fill_synthetic(SEED)  # all DIST U fields, on the device
    names = [f.name for f in FIELDS if f.dist == "M" or f.kind == "ZV"]
    ctx.upload(st, names=names)  # mesh data + one-time precompute + vertical grid
    ctx.sync()


def cpu_baseline(ncells, L, dt, threads, physics=False, transport=False):
    """the oracle (C restatement, -O3, OpenMP) on the host cores: one RK3 step of the
    same workload; kind "port" (the Regent/Legion reference cannot be built or run)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from mpasdyn import build_state as bs
    from mpasdyn import mesh
    m = mesh.icosahedral(LEVEL_OF[ncells])
    if physics:
        m = mesh.zero_based(m)
    st = bs.build_state(m, L, "physical", oracle_fill=lambda s, seed, inc: O.Oracle(s).fill_synthetic(seed, False))
    rdzw, rdzu, fzm, fzp = bs.vertical_grid(st)
    st["rdzw"], st["rdzu"], st["fzm"], st["fzp"] = rdzw, rdzu, fzm, fzp
    o = O.Oracle(st)
    n, t0 = 0, time.perf_counter()
    while n < 8 and (n == 0 or time.perf_counter() - t0 < 10.0):  # a bounded ~10 s sample
        if physics:
            o.mpas_srk3(dt, 1, transport=transport)
        else:
            o.atm_srk3(dt, 1)
        n += 1
    t = (time.perf_counter() - t0) / n
    what = "MPAS-solver " if physics else ""
    what += "RK3 steps with scalar transport" if transport else "RK3 steps"
    return {"value": round(ncells / t / 1e6, 6), "unit": "Mcell-columns/s", "cores": threads, "kind": "port",
            "sample": f"{n} {what} (schedule 0,1,2) of x1.{ncells} x {L} levels by oracle/mpas_oracle.c "
                      f"(-O3, OpenMP {threads} threads), {t:.2f} s per step"}


def pmc_traffic(task, ncells, L, physics=False):
    """per-launch HBM bytes of `task` from a committed rocprofv3 PMC summary, if one
    exists for this configuration (profiles/pmc_x1.<n>_L<L>.json, written by
    tools/pmc_summary.py with the gfx950 FETCH_SIZE correction)"""
    p = os.path.join(REPO, "profiles", f"pmc_{'transport_' if physics else ''}x1.{ncells}_L{L}.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    v = d.get("tasks", {}).get(task)
    return v.get("hbm_bytes_per_launch") if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ncells", type=int, default=163842)
    ap.add_argument("--levels", type=int, default=56)
    ap.add_argument("--exact", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="extra mpas_set_option (A/B runs, e.g. xcd=32)")
    ap.add_argument("--replicas", action="store_true", help="N > 1: full-mesh replicas instead of a decomposition")
    ap.add_argument("--decompose", action="store_true",
                    help="run the decomposed (RCCL halo) path also at N = 1 (a 1-part decomposition)")
    ap.add_argument("--physics", action="store_true",
                    help="the MPAS vertical solver (option physics = 1: 4 acoustic substeps + recover per step)")
    ap.add_argument("--transport", action="store_true",
                    help="physics = 1 plus the monotonic transport of the 8 scalars in every step")
    args = ap.parse_args()
    if args.transport:
        args.physics = True

    # Libraries print banners on stdout from C (RCCL's version lines at communicator
    # creation); the contract is ONE JSON line there: route fd 1 to stderr for the run
    # and print the result through a saved copy of the original stdout.
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", init_method="env://")
    from mpasdyn import lib, roofline
    from mpasdyn import tasks as T

    ncells, L = args.ncells, args.levels
    dt = dt_for(ncells)
    m, st = build_inputs(ncells, L, zero_based=args.physics)
    decomposed = (world > 1 and not args.replicas) or args.decompose
    halo_info = None
    if decomposed:
        from mpasdyn import decomp
        dec = decomp.Decomposition(st, world)
        lst = dec.local_state(rank)
        dims = (*dec.n_local(rank), L)
        ctx = lib.Context(*dims, device=local_rank)
        lib.setup_subdomain(ctx, dec, rank)
        uid = torch.zeros(128, dtype=torch.uint8, device="cuda")
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(lib.rccl_unique_id()), dtype=torch.uint8))
        if dist is not None:
            dist.broadcast(uid, 0)
        lib.halo_rccl(ctx, world, rank, uid.cpu().numpy().tobytes())
        overlap = int(os.environ.get("MPAS_OVERLAP", "1"))
        ctx.set_option("overlap", overlap)
        own = dec.n_owned(rank)
        nint = dec.n_interior(rank)
        halo_info = {"partition": f"{world} contiguous Morton blocks of cells", "owned": list(own),
                     "ghost_frac": [round(1 - o / n, 4) for o, n in zip(own, dims[:3])],
                     "interior_frac": [round(i / max(o, 1), 4) for i, o in zip(nint, own)],
                     "overlap": overlap}
        st = lst
        work_dims = (*own, L)  # what this rank computes
    else:
        dims = (m.nCells, m.nEdges, m.nVertices, L)
        ctx = lib.Context(*dims, device=local_rank)
        work_dims = dims
    ctx.set_option("exact", args.exact)
    ctx.set_option("physics", int(args.physics))
    ctx.set_option("transport", int(args.transport))
    for kv in args.option:
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    upload_inputs(ctx, st)
    hip = Hip()
    stream = ctx.stream()

    for _ in range(args.warmup):
        T.atm_srk3(ctx, dt, 1)
    ctx.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    e0, e1 = hip.event(), hip.event()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hip.record(e0, stream)
    for _ in range(args.steps):
        T.atm_srk3(ctx, dt, 1)
    hip.record(e1, stream)
    ctx.sync()
    torch.cuda.synchronize()
    barrier()
    t_wall = time.perf_counter() - t0
    ev_ms = hip.elapsed_ms(e0, e1)
    ms_step = max(t_wall * 1000.0, ev_ms) / args.steps
    if dist is not None:
        t = torch.tensor([ms_step], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms_step = float(t.item())

    # per-task device times (HIP events bracketing every task on the task stream)
    ctx.timing(True)
    ctx.timing_reset()
    n_prof = 2
    for _ in range(n_prof):
        T.atm_srk3(ctx, dt, 1)
    ctx.sync()
    rep = ctx.timing_report()
    ctx.timing(False)
    kw_of = {"atm_compute_dyn_tend_work[rk0]": ("atm_compute_dyn_tend_work", {"rk_step": 0}),
             "atm_compute_dyn_tend_work[rk>0]": ("atm_compute_dyn_tend_work", {"rk_step": 1}),
             "atm_recover_large_step_variables_work": ("atm_recover_large_step_variables_work", {"rk_step": 2})}
    tasks_out = {}
    if args.physics:  # the acoustic task's MPAS form also updates ru_p / ruAvg
        kw_of["atm_advance_acoustic_step_work"] = ("atm_advance_acoustic_step_work", {"physics": 1})
    for name, (calls, ms) in rep.items():
        task, kw = kw_of.get(name, (name, {}))
        b = roofline.b_alg(task, work_dims, **kw)
        avg = ms / calls
        tasks_out[name] = {"launches_per_step": calls // n_prof, "avg_ms": round(avg, 4),
                           "b_alg_GB": round(b / 1e9, 4), "GBs": round(b / (avg * 1e-3) / 1e9, 1)}
        tr = pmc_traffic(name, ncells, L, args.physics) if not decomposed else None
        if tr:  # SURVEY §8.5 metric 2: measured (FETCH + WRITE) bytes over this run's launch time
            tasks_out[name]["hbm_GB_measured"] = round(tr / 1e9, 4)
            tasks_out[name]["hbm_frac_measured"] = round(tr / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    dom = max(tasks_out, key=lambda k: tasks_out[k]["avg_ms"] * tasks_out[k]["launches_per_step"])
    dt_ = tasks_out[dom]
    task, kw = kw_of.get(dom, (dom, {}))
    traffic = pmc_traffic(dom, ncells, L, args.physics) if not decomposed else None
    traffic = round(traffic / 1e9, 4) if traffic else None
    roof = {"bound": "hbm", "kernel": dom, "achieved": dt_["GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(dt_["GBs"] / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_unit": "GB/launch",
            "b_alg_per_launch_GB": dt_["b_alg_GB"], "avg_launch_ms": dt_["avg_ms"],
            "traffic_frac": dt_.get("hbm_frac_measured")}
    b_step = roofline.b_alg_step(work_dims, 1, int(args.physics), int(args.transport))
    step_gbs = b_step / (ms_step * 1e-3) / 1e9

    value = (1 if decomposed else world) * ncells / (ms_step * 1e-3) / 1e6
    if decomposed:
        ex, fl = lib.halo_stats(ctx)
        halo_info["exchanges_per_step"] = round(ex / (args.warmup + args.steps + n_prof), 2)
        halo_info["fields_per_step"] = round(fl / (args.warmup + args.steps + n_prof), 2)
    out = {"metric": METRIC, "value": round(value, 3), "unit": "Mcell-columns/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
           "scaling": "strong" if decomposed else "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": f"x1.{ncells} x {L} levels, atm_srk3 (3 dyn_tend rk 0/1/2, " +
                                  ("4 acoustic substeps + recover (MPAS vertical solver)" if args.physics
                                   else "7 acoustic substeps") +
                                  (", monotonic transport of 8 scalars" if args.transport else "") + ")",
                      "nCells": ncells, "nEdges": m.nEdges, "nVertices": m.nVertices, "nVertLevels": L,
                      "dt": dt, "parallelism": (f"decomposed{world}" if decomposed else
                                                 f"replicas{world}" if world > 1 else "single-gpu"),
                      "exact": args.exact, "physics": int(args.physics), "transport": int(args.transport)},
           "step_b_alg_GB": round(b_step / 1e9, 3), "step_achieved_GBs": round(step_gbs, 1),
           "roofline": roof, "tasks": tasks_out}
    if halo_info:
        out["halo"] = halo_info
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count())))
        out["cpu_baseline"] = cpu_baseline(ncells, L, dt, threads, args.physics, args.transport)
    elif rank == 0:
        out["cpu_baseline"] = None
    ctx.close()
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
