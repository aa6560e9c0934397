#!/usr/bin/env python3
"""Benchmark of the RK3 dynamics hot path (atm_srk3, rk_timestep.rg:361-500) on MI355X.

Metric (BASELINE.json): Mcell-columns/s per RK3 step at x1.163842 x 56 levels, plus the
achieved HBM bandwidth of the dominant task against the 8 TB/s roofline.

One step = one atm_srk3 call: setup, moist, 2x vert_imp, 3x dyn_tend (rk_step 0,1,2 --
the MPAS schedule of SURVEY §8.5), 3x smlstep, 7x acoustic + 7x divergence damping,
3x solve_diagnostics, substep_finish (28 tasks of the reference schedule; the library's
fusions and option ntu's liveness launch fewer kernels for the same results -- every field
after the step is bit-identical).  Inputs are resident in HBM before the
timed region: the x1.163842 icosahedral mesh (mpasdyn.mesh) with its one-time
precompute uploaded from the host, and the 3-D state filled on the device by the
seeded generator (data: synthetic, seed 20211015).

    python bench.py [--gpus N --steps K --warmup W]

N > 1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) the ranks are
the launcher's and WORLD_SIZE must equal N; without it bench.py starts the N rank
processes itself (children with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT, before
any GPU call; rank 0's stdout is the JSON line).  The x1.163842 mesh is split into N
subdomains (mpasdyn/decomp.py: contiguous blocks of the Morton-ordered cells,
edges/vertices with their first cell/edge, ghosts = everything an owned entity reaches
through an index array), and the ranks exchange halos with RCCL send/recv before every
kernel that gathers a field another rank wrote (csrc/mpas_halo.h).  Total work is fixed
("scaling": "strong"); `value` = global cell columns / step time.  `--replicas` instead
runs a full-mesh replica per rank (weak scaling, no collective).

roofline: the task with the largest device time per step (atm_compute_dyn_tend_work, the
north-star kernel; its rk_step 0 and rk_step > 0 launches are one Regent task),
achieved = its algorithmic bytes per step (mpasdyn/roofline.py) / its
device time per step (HIP events on the task stream), i.e. the launch-weighted average;
traffic = its HBM bytes per launch from rocprofv3 FETCH_SIZE and WRITE_SIZE passes over
this same workload, run by this script before it touches the GPU (--traffic auto).

Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import shutil
import socket
import statistics
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mpas-regent_amd"))

import numpy as np  # noqa: E402

METRIC = "Mcell-columns/sec per RK3 step; achieved HBM GB/s; x1.163842×56L"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak
LEVEL_OF = {2562: 4, 10242: 5, 40962: 6, 163842: 7, 655362: 8}
SEED = 20211015
NORTH_STAR = "atm_compute_dyn_tend_work"


class Hip:
    """the few HIP runtime calls the timing needs (events on the library's stream, device
    synchronisation).  Bound after libmpasdyn is loaded, by its soname: the dynamic loader
    then returns the HIP runtime the library already runs on (its RUNPATH's), never a
    second one (INTEGRATION.md "One HIP runtime per process")."""

    def __init__(self):
        from mpasdyn import lib
        lib.load()
        self.h = ctypes.CDLL("libamdhip64.so.7")
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

    def device_sync(self):
        assert self.h.hipDeviceSynchronize() == 0

    def device_count(self):
        n = ctypes.c_int(0)
        assert self.h.hipGetDeviceCount(ctypes.byref(n)) == 0
        return int(n.value)

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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(ncells, L, dt, threads, physics=False, transport=False, budget_s=20.0):
    """the oracle (C restatement, -O3, OpenMP) on the host cores, RK3 steps of the same
    workload; kind "port" (the Regent/Legion reference cannot be built or run).  Two
    untimed warm-up steps, then steps timed one by one until `budget_s` (at least 3,
    at most 20); value from the median step."""
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

    def step():
        if physics:
            o.mpas_srk3(dt, 1, transport=transport, physics=int(physics))
        else:
            o.atm_srk3(dt, 1)

    warm = 2
    for _ in range(warm):
        step()
    times, t0 = [], time.perf_counter()
    while len(times) < 20 and (len(times) < 3 or time.perf_counter() - t0 < budget_s):
        t1 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t1)
    t = statistics.median(times)
    what = {0: "", 1: "MPAS-solver ", 2: "MPAS-dynamics "}[int(physics)]
    what += "RK3 steps with scalar transport" if transport else "RK3 steps"
    return {"value": round(ncells / t / 1e6, 6), "unit": "Mcell-columns/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "omp_num_threads": threads, "nproc": os.cpu_count(),
            "sample": f"median of {len(times)} {what} (schedule 0,1,2) after {warm} warm-up steps, x1.{ncells} x {L} "
                      f"levels, oracle/mpas_oracle.c (-O3, OpenMP {threads} threads): {t:.3f} s per step "
                      f"(min {min(times):.3f}, max {max(times):.3f}); bounded to ~{budget_s:.0f} s of CPU time, "
                      f"fewer than the 20 steps SURVEY §8.5 asks when a step is slower than {budget_s / 20:.1f} s"}


# ------------------------------------------------------------------ process launch
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def free_port_range(n):
    """a base port with n free consecutive ports (the socket halo transport: rank r on base + r)"""
    for _ in range(50):
        base = free_port()
        if base + n >= 65535:
            continue
        ok = True
        for q in range(base, base + n):
            t = socket.socket()
            try:
                t.bind(("127.0.0.1", q))
            except OSError:
                ok = False
            finally:
                t.close()
            if not ok:
                break
        if ok:
            return base
    raise RuntimeError("no free port range")


class Watchdog:
    """a bounded wait on a blocking call that cannot time out by itself (ncclCommInitRank, the
    first exchange of the first step): unless cancelled within `seconds`, the rank prints a
    named error and exits with status 3 -- the launcher (torchrun, or spawn_ranks) then ends
    the other ranks, instead of the job hanging until an outer limit kills it"""

    def __init__(self, seconds, what, rank):
        import threading
        self.what, self.rank = what, rank
        self.t = threading.Timer(seconds, self._fire, args=(seconds,))
        self.t.daemon = True
        self.t.start()

    def _fire(self, seconds):
        print(f"bench.py rank {self.rank}: {self.what} did not complete within {seconds:.0f} s "
              f"(a rank missing or a transport that cannot connect); exiting", file=sys.stderr, flush=True)
        os._exit(3)

    def cancel(self):
        self.t.cancel()


def dump_rows(path, ctx, st, gids, steps, extra):
    """tests (--dump): one 64-bit fingerprint per owned row of every fp64 field -- the row's
    bits (-0.0 as +0.0, every NaN as one NaN) under a fixed linear hash -- with the rows'
    global ids, so that the owned parts of N ranks can be compared with one context bit for
    bit without moving the fields themselves (tests/test_gpu_bench.py)"""
    from mpasdyn.registry import FIELDS
    from mpasdyn.state import HostState
    out = {f"gid_{k}": np.asarray(v, dtype=np.int64) for k, v in gids.items()}
    rng = np.random.default_rng(12345)
    for f in FIELDS:
        if f.entity is None or f.dtype != np.float64:
            continue
        got = HostState(*st.dims(), names=[f.name])  # (one field at a time: host memory)
        ctx.download(got)
        a = np.asarray(got.arrays[f.name])[:len(gids[f.entity])]
        a = np.where(np.isnan(a), np.nan, a) + 0.0  # (canonical NaN, -0.0 -> +0.0)
        bits = np.ascontiguousarray(a.reshape(len(a), -1)).view(np.uint64)
        mult = rng.integers(1, 2**63, size=bits.shape[1], dtype=np.uint64) | np.uint64(1)
        with np.errstate(over="ignore"):
            out[f.name] = (bits * mult[None, :]).sum(axis=1, dtype=np.uint64)
    out["steps"] = np.int64(steps)
    for k, v in extra.items():
        out[k] = np.asarray(v)
    np.savez(path, **out)


def spawn_ranks(n, argv):
    """start N rank processes of this script (no GPU touched here); rank 0 inherits
    stdout (the JSON line), the others write theirs to stderr.  Returns the exit code."""
    port, rdzv = free_port(), free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MPAS_RDZV_PORT=str(rdzv))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                c = p.poll()
                if c is None:
                    continue
                pending.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    for q in pending:  # one rank failed: the others would wait forever
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


# ------------------------------------------------------------------ live HBM traffic
def measure_traffic(args):
    """run this workload (one RK3 step, no warm-up) under `rocprofv3 --pmc FETCH_SIZE`
    and under `--pmc WRITE_SIZE` (separate passes, MI355X_MICROARCH.md) in child
    processes, before this process touches the GPU; returns {timing key: HBM bytes per
    step} and a note, or (None, reason)."""
    from mpasdyn import pmc
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "1", "--warmup", "0",
             "--ncells", str(args.ncells), "--levels", str(args.levels), "--exact", str(args.exact)]
    child += [f"--option={o}" for o in args.option]
    if args.physics:
        child.append(f"--physics={args.physics}")
    if args.transport:
        child.append("--transport")
    res = {}
    tmp = tempfile.mkdtemp(prefix="mpas_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = ["timeout", "-s", "KILL", "240", prof, "--pmc", counter, "-d", d, "-o", "pmc",
                   "--output-format", "csv", "--"] + child
            p = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, cwd=REPO)
            if p.returncode != 0:
                return None, f"rocprofv3 --pmc {counter} exited {p.returncode}: {p.stderr[-300:]}"
            res[counter] = pmc.read_counter(d, counter)
    except Exception as e:  # noqa: BLE001 -- traffic is optional; report why it is null
        return None, f"{type(e).__name__}: {e}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    m_cells = args.ncells
    m_edges = 3 * (m_cells - 2)
    wfac = pmc.write_factor(res["WRITE_SIZE"], m_cells, m_edges, args.levels, int(args.physics or 0))
    if wfac is None:
        return None, "WRITE_SIZE calibration kernels missing"
    by = pmc.bytes_per_step(pmc.drop_calibration(res["FETCH_SIZE"]), pmc.drop_calibration(res["WRITE_SIZE"]), 1,
                            wfac)
    return by, (f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of 1 RK3 step of this workload; "
                f"fetch x{pmc.FETCH_FACTOR} (gfx950), write x{wfac:.3f} (calibrated on the setup copies)")


def pmc_child(args):
    """the workload rocprofv3 counts: 1 RK3 step after upload, then one setup task alone"""
    from mpasdyn import lib
    from mpasdyn import tasks as T
    m, st = build_inputs(args.ncells, args.levels, zero_based=args.physics)
    ctx = lib.Context(m.nCells, m.nEdges, m.nVertices, args.levels, device=0)
    ctx.set_option("exact", args.exact)
    ctx.set_option("physics", int(args.physics))
    ctx.set_option("transport", int(args.transport))
    for kv in args.option:
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    upload_inputs(ctx, st)
    dt = dt_for(args.ncells)
    for _ in range(args.steps):
        T.atm_srk3(ctx, dt, 1)
    # the WRITE_SIZE calibration: the setup task's pure copies, run alone (the step may
    # have fused them into another launch); measure_traffic drops this dispatch again
    T.atm_rk_integration_setup(ctx)
    ctx.sync()
    ctx.close()


# ------------------------------------------------------------------ roofline
def task_table(rep, work_dims, n_prof, physics, ddx=False):
    """per timing key (a task, split by the arguments that change its read/write set)
    and aggregated per Regent task: launches and device ms per step, B_alg per step"""
    from mpasdyn import roofline
    kw_of = {"atm_compute_dyn_tend_work[rk0]": {"rk_step": 0}, "atm_compute_dyn_tend_work[rk>0]": {"rk_step": 1},
             "atm_advance_acoustic_step_work[ss0]": {"small_step": 0},
             "atm_advance_acoustic_step_work[ss>0]": {"small_step": 1},
             "atm_advance_acoustic_step_work[ss0+damp]": {"small_step": 0, "damp": True},
             "atm_rk_integration_setup[+moist+vert_imp]": {"fused": True},
             "atm_rk_integration_setup[cells+moist+vert_imp]": {"fused": True, "copy": True},
             "atm_compute_dyn_tend_work[rk0+copy]": {"rk_step": 0, "copy": True},
             "atm_compute_dyn_tend_work[rk>0+copy]": {"rk_step": 1, "copy": True},
             "atm_advance_acoustic_step_work[ss0+sml]": {"small_step": 0, "sml": True},
             "atm_advance_acoustic_step_work[ss0+smlS]": {"small_step": 0, "sml": True, "smls": True},
             "atm_advance_acoustic_step_work[ss0+smlS+damp]": {"small_step": 0, "damp": True, "sml": True, "smls": True},
             "atm_set_smlstep_pert_variables_work[flux]": {"part": "flux"},
             "atm_compute_solve_diagnostics[vc]": {"part": "vc"}, "atm_compute_solve_diagnostics[e]": {"part": "e"},
             "hfuse[damp+solve_vc]": {"pair": "damp+solve_vc"}, "hfuse[solve_e+finish]": {"pair": "solve_e+finish"},
             "hfuse[solve_e-v+finish]": {"pair": "solve_e-v+finish"},
             "hfuse[solve_e+finish-rz]": {"pair": "solve_e+finish-rz"},
             "hfuse[solve_e-v+finish-rz]": {"pair": "solve_e-v+finish-rz"},
             "atm_rk_dynamics_substep_finish[-rz]": {"norz": True},
             "atm_compute_solve_diagnostics[e-v]": {"part": "e"}, "atm_compute_solve_diagnostics[-v]": {},
             "atm_compute_solve_diagnostics[live]": {"live": True},
             "hfuse[solve_e+vert_imp]": {"pair": "solve_e+vert_imp"},
             "hfuse[acoustic+solve_vc]": {"pair": "acoustic+solve_vc"},
             "hfuse[acoustic-st+solve_vc]": {"pair": "acoustic-st+solve_vc"},
             "hfuse[solve_e+dyn_A]": {"pair": "solve_e+dyn_A"},
             "hfuse[solve_e+vert_imp+dyn_A]": {"pair": "solve_e+vert_imp+dyn_A"},
             "atm_compute_dyn_tend_work[rk>0-A]": {"rk_step": 1, "noA": True},
             "atm_compute_dyn_tend_work[rk0-A]": {"rk_step": 0, "noA": True},
             "atm_compute_dyn_tend_work[rk0+copy-A]": {"rk_step": 0, "copy": True, "noA": True},
             "atm_compute_dyn_tend_work[rk>0+copy-A]": {"rk_step": 1, "copy": True, "noA": True},
             "hfuse[setup+dyn_A]": {"pair": "setup+dyn_A"},
             "hfuse[setup+dyn_A+sml_flux]": {"pair": "setup+dyn_A+sml_flux"},
             "atm_advance_acoustic_step_work[ss0+sml+damp]": {"small_step": 0, "damp": True, "sml": True},
             "atm_advance_acoustic_step_work[ss>0+damp]": {"small_step": 1, "damp": True},
             "atm_recover_large_step_variables_work[rk<2]": {"rk_step": 0},
             "atm_recover_large_step_variables_work[rk2]": {"rk_step": 2},
             "atm_recover_large_step_variables_work[rk<2-avg]": {"rk_step": 0, "navg": True},
             "atm_advance_scalars_mono[save]": {"save": True},
             # (option mdamp: the stage's last divergence damping in the recover edge kernel)
             "atm_recover_large_step_variables_work[rk<2-avg+damp]": {"rk_step": 0, "navg": True, "damp": True},
             "atm_recover_large_step_variables_work[rk1-avg+damp]": {"rk_step": 1, "navg": True, "damp": True},
             "atm_recover_large_step_variables_work[rk1-avg]": {"rk_step": 1, "navg": True},
             "atm_recover_large_step_variables_work[rk<2+damp]": {"rk_step": 0, "damp": True},
             "atm_recover_large_step_variables_work[rk2+damp]": {"rk_step": 2, "damp": True}}
    def dyn_kw(name):  # atm_compute_dyn_tend_work[rk0|rk>0 (+copy) (+d4o) (+d4i) (-A)] (mpas_ctx.cpp srk3)
        tag = name[name.index("[") + 1:-1]
        kw = {"rk_step": 0 if tag.startswith("rk0") else 1}
        if "+copy" in tag:
            kw["copy"] = True
        if "+d4o" in tag:
            kw["defer_out"] = True
        if "+ntu" in tag:  # (option ntu: a stage before the step's last, its dead tendencies not formed)
            kw["ntu"] = True
        if "+v" in tag:
            kw["store_v"] = True
        if "+ru" in tag:  # (option mru: the first substep's ru_p / ruAvg stored here)
            kw["ru"] = True
        if "+sml" in tag:  # (option msml: the stage's set_smlstep in E)
            kw["smle"] = True
        if tag.endswith("-A"):
            kw["noA"] = True
        return kw

    variants, tasks = {}, {}
    for name, (calls, ms) in rep.items():
        task = name.split("[")[0]
        # ("-st]": option ntu's acoustic launch that stores no acoustic state, the last substep of a stage
        # before the step's last)
        # ("-ru]", outermost: option mru, the first substep's ru_p / ruAvg stored by dyn_tend; "-ww]": the MPAS
        # forms' counterpart of "-st", wwAvg alone unstored)
        base, nbc = (name[:-4] + "]", True) if name.endswith("-bc]") else (name, False)  # (ntu: b_tri / c_tri)
        base, rud = (base[:-4] + "]", True) if base.endswith("-ru]") else (base, False)
        base, nww = (base[:-4] + "]", True) if base.endswith("-ww]") else (base, False)
        base, nst = (base[:-4] + "]", True) if base.endswith("-st]") else (base, False)
        if task == NORTH_STAR and "[" in name:
            kw = dyn_kw(name)
        elif base.endswith("-old]"):  # a fused acoustic launch that leaves rtheta_pp_old (mpas_ctx.cpp)
            kw = dict(kw_of.get(base[:-5] + "]", {}), wold=False)
        else:
            kw = dict(kw_of.get(base, {}))
        if nst:
            kw["nst"] = True
        if nww:
            kw["nww"] = True
        if rud:
            kw["rudone"] = True
        if nbc:
            kw["nbc"] = True
        if ddx and (task == "atm_advance_acoustic_step_work" or name in ("hfuse[acoustic+solve_vc]",
                                                                         "hfuse[acoustic-st+solve_vc]")):
            kw["ddx"] = True  # (option smlsum: the acoustic launches read rw_save - rw from X_Dd)
        if physics and task == "atm_advance_acoustic_step_work":
            kw["physics"] = 1  # the acoustic task's MPAS form also updates ru_p / ruAvg
        if physics == 2 and task in ("atm_rk_integration_setup", "atm_compute_moist_coefficients",
                                     "atm_compute_dyn_tend_work", "atm_set_smlstep_pert_variables_work",
                                     "atm_compute_solve_diagnostics", "atm_rk_dynamics_substep_finish"):
            kw["physics"] = 2  # the MPAS dynamics' read/write sets
        b = roofline.b_alg(task, work_dims, **kw)
        avg = ms / calls
        n = calls / n_prof
        variants[name] = {"launches_per_step": round(n, 3), "avg_ms": round(avg, 4), "b_alg_GB": round(b / 1e9, 4),
                          "GBs": round(b / (avg * 1e-3) / 1e9, 1)}
        if kw.get("copy") and task == NORTH_STAR:  # the setup copies fusecopy moved in
            variants[name]["b_alg_GB_excl_fusecopy"] = round(roofline.b_alg(task, work_dims, **dict(kw, copy=False)) / 1e9, 4)
        t = tasks.setdefault(task, {"launches_per_step": 0.0, "ms_per_step": 0.0, "b_alg_GB_per_step": 0.0})
        t["launches_per_step"] += n
        t["ms_per_step"] += n * avg
        t["b_alg_GB_per_step"] += n * b / 1e9
    for name, t in tasks.items():
        t["avg_ms"] = round(t["ms_per_step"] / t["launches_per_step"], 4)
        t["b_alg_GB"] = round(t["b_alg_GB_per_step"] / t["launches_per_step"], 4)  # per launch
        t["GBs"] = round(t["b_alg_GB_per_step"] / (t["ms_per_step"] * 1e-3), 1)
        t["frac"] = round(t["GBs"] / HBM_PEAK_GBS, 4)
        t["launches_per_step"] = round(t["launches_per_step"], 3)
        t["ms_per_step"] = round(t["ms_per_step"], 4)
        t["b_alg_GB_per_step"] = round(t["b_alg_GB_per_step"], 4)
        vs = {k[len(name):]: v for k, v in variants.items() if k.split("[")[0] == name and "[" in k}
        if vs:
            t["variants"] = vs
    return tasks


def frac_excl_copy(t):
    """the task's B_alg fraction without the bytes of the setup copies (ru_save = ru, u_2 = u) that
    option fusecopy moved into its rk_step 0 launch"""
    vs = (t.get("variants") or {}).values()
    b = sum(v["launches_per_step"] * v.get("b_alg_GB_excl_fusecopy", v["b_alg_GB"]) for v in vs) if vs else t["b_alg_GB_per_step"]
    return round(b / (t["ms_per_step"] * 1e-3) / HBM_PEAK_GBS, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ncells", type=int, default=163842)
    ap.add_argument("--levels", type=int, default=56)
    ap.add_argument("--exact", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of oracle steps in the cpu_baseline leg")
    ap.add_argument("--traffic", choices=["auto", "off"], default="auto",
                    help="auto: rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this workload (N = 1, rank 0)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-run", action="store_true", help="print each rank's launch environment and exit")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="extra mpas_set_option (A/B runs, e.g. xcd=32)")
    ap.add_argument("--replicas", action="store_true", help="N > 1: full-mesh replicas instead of a decomposition")
    ap.add_argument("--halo", choices=["rccl", "socket"], default="rccl",
                    help="socket: the host-staged TCP transport, ranks sharing the visible GPUs -- a rehearsal of "
                         "the multi-rank flow on one GPU, not a measurement")
    ap.add_argument("--decompose", action="store_true",
                    help="run the decomposed (RCCL halo) path also at N = 1 (a 1-part decomposition)")
    ap.add_argument("--physics", type=int, nargs="?", const=1, default=0, choices=[0, 1, 2],
                    help="1: the MPAS vertical solver (4 acoustic substeps + recover per step); 2: also the MPAS "
                         "dynamics (every quirk fixed)")
    ap.add_argument("--transport", action="store_true",
                    help="physics = 1 plus the monotonic transport of the 8 scalars in every step")
    ap.add_argument("--dump", metavar="DIR", help=argparse.SUPPRESS)  # (tests: per-row fingerprints, see dump_rows)
    ap.add_argument("--init-timeout", type=float, default=float(os.environ.get("MPAS_INIT_TIMEOUT", "300")),
                    help="seconds the communicator set-up and the first (exchanging) step may take before the rank "
                         "exits non-zero with a named error instead of hanging")
    args = ap.parse_args()
    if args.transport and not args.physics:
        args.physics = 1
    if args.pmc_child:
        return pmc_child(args)

    # ranks: the launcher's (torch.distributed.run) or our own children
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
            return 2
    elif args.gpus > 1:
        return spawn_ranks(args.gpus, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    from mpasdyn.rendezvous import Rendezvous
    if args.dry_run:
        # the launch environment plus one round of the host rendezvous (unique-id
        # broadcast, max, barrier) -- with no GPU call and no torch
        rv = Rendezvous(rank, world, os.environ.get("MASTER_ADDR", "127.0.0.1")) if world > 1 else None
        uid = rv.bcast(b"uid-from-rank-0" if rank == 0 else None) if rv else b""
        mx = rv.allreduce_max(float(rank)) if rv else 0.0
        if rv:
            rv.barrier()
            rv.close()
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world_size": world, "gpus": args.gpus,
                          "master": f"{os.environ.get('MASTER_ADDR', '')}:{os.environ.get('MASTER_PORT', '')}",
                          "bcast": uid.decode(), "max_rank": mx, "torch_loaded": "torch" in sys.modules}),
              flush=True)
        return 0

    # live traffic first: the profiled children start before this process touches the GPU
    traffic_by, traffic_note = None, "off"
    if args.traffic == "auto" and world == 1 and rank == 0 and not args.decompose:
        traffic_by, traffic_note = measure_traffic(args)

    # Libraries print banners on stdout from C (RCCL's version lines at communicator
    # creation); the contract is ONE JSON line there: route fd 1 to stderr for the run
    # and print the result through a saved copy of the original stdout.
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    # ranks meet over a plain TCP rendezvous (mpasdyn/rendezvous.py): no torch in this
    # process, so the one HIP runtime is the library's
    rv = Rendezvous(rank, world, os.environ.get("MASTER_ADDR", "127.0.0.1")) if world > 1 else None
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
        device = local_rank if args.halo == "rccl" else local_rank % Hip().device_count()
        ctx = lib.Context(*dims, device=device)
        lib.setup_subdomain(ctx, dec, rank)
        if args.halo == "socket":  # rank r listens on base + r (rank 0 picks the range)
            base = str(free_port_range(world)).encode() if rank == 0 else None
            if rv is not None:
                base = rv.bcast(base)
            lib.halo_socket(ctx, world, rank, "127.0.0.1", int(base.decode()))
        else:
            uid = lib.rccl_unique_id() if rank == 0 else None
            if rv is not None:
                uid = rv.bcast(uid)
            wd = Watchdog(args.init_timeout, "ncclCommInitRank", rank)
            lib.halo_rccl(ctx, world, rank, uid)
            wd.cancel()
        overlap = int(os.environ.get("MPAS_OVERLAP", "1"))
        ctx.set_option("overlap", overlap)
        own = dec.n_owned(rank)
        nint = dec.n_interior(rank)
        halo_info = {"partition": f"{world} contiguous blocks of the curve-ordered cells (cube-face Hilbert)",
                     "transport": args.halo if args.halo == "rccl" else "socket (host-staged TCP rehearsal, not a measurement)",
                     "owned": list(own),
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

    # (the first step makes the first halo exchanges: bounded like the communicator set-up)
    wd = Watchdog(args.init_timeout, "the first RK3 step (its halo exchanges)", rank) if decomposed else None
    for i in range(args.warmup):
        T.atm_srk3(ctx, dt, 1)
        if i == 0 and wd is not None:
            ctx.sync()
            wd.cancel()
            wd = None
    ctx.sync()

    def barrier():
        if rv is not None:
            rv.barrier()

    # K timed steps, bracketed by barrier + device synchronisation on both sides; one HIP
    # event between consecutive steps on the task stream gives the per-step device times
    # (the median step), the wall clock the whole region
    evs = [hip.event() for _ in range(args.steps + 1)]
    barrier()
    hip.device_sync()
    t0 = time.perf_counter()
    hip.record(evs[0], stream)
    for i in range(args.steps):
        T.atm_srk3(ctx, dt, 1)
        hip.record(evs[i + 1], stream)
        if wd is not None:  # (no warm-up: the first timed step made the first exchanges)
            ctx.sync()
            wd.cancel()
            wd = None
    ctx.sync()
    hip.device_sync()
    barrier()
    if args.dump:  # (after the timed steps, before the per-task timing steps)
        os.makedirs(args.dump, exist_ok=True)
        if decomposed:
            gids = {k: dec.owned[rank][k] for k in ("cell", "edge", "vertex")}
            ex = lib.halo_stats(ctx)[0]
        else:
            gids = {"cell": np.arange(m.nCells), "edge": np.arange(m.nEdges), "vertex": np.arange(m.nVertices)}
            ex = 0
        dump_rows(os.path.join(args.dump, f"rank{rank}.npz"), ctx, st, gids, args.warmup + args.steps,
                  {"exchanges": ex, "world": world})
        barrier()
    t_wall = time.perf_counter() - t0
    step_ms = [hip.elapsed_ms(evs[i], evs[i + 1]) for i in range(args.steps)]
    ms_median = statistics.median(step_ms)
    ms_mean = max(t_wall * 1000.0, sum(step_ms)) / args.steps
    if rv is not None:  # the slowest rank sets the job's step time
        ms_median = rv.allreduce_max(ms_median)
        ms_mean = rv.allreduce_max(ms_mean)
    ms_step = ms_median

    # per-task device times (HIP events bracketing every task on the task stream)
    ctx.timing(True)
    ctx.timing_reset()
    n_prof = 2
    for _ in range(n_prof):
        T.atm_srk3(ctx, dt, 1)
    ctx.sync()
    rep = ctx.timing_report()
    ctx.timing(False)
    smls = (bool(ctx.get_option("fusedamp_active")) and bool(ctx.get_option("fusesml")) and
            bool(ctx.get_option("smlsum")) and not args.exact and not args.physics)
    tasks_out = task_table(rep, work_dims, n_prof, args.physics, ddx=smls)
    if traffic_by:
        for name, t in tasks_out.items():
            keys = [k for k in traffic_by if k.split("[")[0] == name]
            if keys:  # SURVEY §8.5 metric 2: measured (FETCH + WRITE) bytes over this run's device time
                b = sum(sum(traffic_by[k]) for k in keys)
                t["hbm_GB_measured_per_step"] = round(b / 1e9, 4)
                t["hbm_frac_measured"] = round(b / (t["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    dom = max(tasks_out, key=lambda k: tasks_out[k]["ms_per_step"])
    ns = tasks_out[NORTH_STAR]
    traffic = None
    if "hbm_GB_measured_per_step" in ns:
        traffic = round(ns["hbm_GB_measured_per_step"] / ns["launches_per_step"], 4)
    roof = {"bound": "hbm", "kernel": NORTH_STAR, "achieved": ns["GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ns["frac"], "traffic": traffic, "traffic_unit": "GB/launch",
            "traffic_over_b_alg": round(traffic / ns["b_alg_GB"], 3) if traffic else None,
            "traffic_frac": ns.get("hbm_frac_measured"), "traffic_source": traffic_note,
            "b_alg_per_launch_GB": ns["b_alg_GB"], "avg_launch_ms": ns["avg_ms"],
            "launches_per_step": ns["launches_per_step"], "ms_per_step": ns["ms_per_step"],
            "frac_excl_fusecopy": frac_excl_copy(ns), "variants": ns.get("variants"), "dominant_task": dom,
            "note": "achieved = B_alg per step / device time per step of the task (launch-weighted average of its "
                    "rk_step 0 and rk_step > 0 launches); frac = achieved / peak"}
    fused = bool(ctx.get_option("fusedamp_active"))
    fsetup = bool(ctx.get_option("fusesetup"))
    fsml = fused and bool(ctx.get_option("fusesml")) and not args.physics
    fcopy = fsetup and bool(ctx.get_option("fusecopy"))  # (decomposed and MPAS forms too, as srk3 does)
    d4 = bool(ctx.get_option("defer4")) and not args.physics
    ntu = bool(ctx.get_option("ntu"))  # (the MPAS forms: the dead diagnostics and averages only)
    mdamp = bool(ctx.get_option("mdamp")) and bool(args.physics)
    # (option trsave: scalars_save folded into the transport, undecomposed with the default transport kernels)
    trsave = bool(args.transport) and bool(ctx.get_option("trsave")) and not decomposed and not any(
        ctx.get_option(o) for o in ("trtile", "tredge", "trsu"))
    mru = bool(ctx.get_option("mru")) and int(args.physics) == 2 and not args.exact
    msml = bool(ctx.get_option("msml")) and int(args.physics) == 2
    b_step = roofline.b_alg_step(work_dims, 1, int(args.physics), int(args.transport), fused, fsetup, fsml, fcopy, d4,
                                 smls, ntu, mdamp, trsave, mru, msml)
    step_gbs = b_step / (ms_step * 1e-3) / 1e9

    value = (1 if decomposed else world) * ncells / (ms_step * 1e-3) / 1e6
    if decomposed:
        ex, fl = lib.halo_stats(ctx)
        halo_info["exchanges_per_step"] = round(ex / (args.warmup + args.steps + n_prof), 2)
        halo_info["fields_per_step"] = round(fl / (args.warmup + args.steps + n_prof), 2)
    out = {"metric": METRIC, "value": round(value, 3), "unit": "Mcell-columns/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
           "ms_per_step_stat": f"median of {args.steps} per-step HIP-event times on the task stream, max over ranks "
                               f"(SURVEY §8.5)", "ms_per_step_mean": round(ms_mean, 4),
           "ms_per_step_min_max": [round(min(step_ms), 4), round(max(step_ms), 4)], "higher_is_better": True,
           "scaling": "strong" if decomposed else "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": f"x1.{ncells} x {L} levels, atm_srk3 (3 dyn_tend rk 0/1/2, " +
                                  ({1: "4 acoustic substeps + recover (MPAS vertical solver)",
                                    2: "4 acoustic substeps + recover, MPAS dynamics (physics 2)"}.get(args.physics,
                                                                                     "7 acoustic substeps")) +
                                  (", monotonic transport of 8 scalars" if args.transport else "") + ")",
                      "nCells": ncells, "nEdges": m.nEdges, "nVertices": m.nVertices, "nVertLevels": L,
                      "dt": dt, "parallelism": (f"decomposed{world}" if decomposed else
                                                 f"replicas{world}" if world > 1 else "single-gpu"),
                      "exact": args.exact, "physics": int(args.physics), "transport": int(args.transport),
                      "graph": ctx.get_option("graph") if not decomposed else 0, "fusedamp": int(fused), "fusesetup": int(fsetup), "fusecopy": int(fcopy), "smlsum": int(smls),
                      "fusesml": int(fsml), "defer4": int(d4), "ntu": int(ntu), "mdamp": int(mdamp), "trsave": int(trsave), "mru": int(mru), "msml": int(msml), "tmedge": int(fused and bool(ctx.get_option("tmedge"))),
                      "hfuse": int(bool(ctx.get_option("hfuse_active")))},
           "step_b_alg_GB": round(b_step / 1e9, 3), "step_achieved_GBs": round(step_gbs, 1),
           "roofline": roof, "tasks": tasks_out}
    if halo_info:
        out["halo"] = halo_info
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # all the host cores this process may use: the OMP_NUM_THREADS pin when the
        # environment sets one (the GPU box pins 16, its CPU share per GPU), else nproc
        pin = os.environ.get("OMP_NUM_THREADS")
        threads = int(pin) if pin else (len(os.sched_getaffinity(0)) or os.cpu_count())
        if not pin:
            os.environ["OMP_NUM_THREADS"] = str(threads)
        out["cpu_baseline"] = cpu_baseline(ncells, L, dt, threads, args.physics, args.transport, args.cpu_budget)
        out["cpu_baseline"]["threads_from"] = "OMP_NUM_THREADS (environment pin)" if pin else "sched_getaffinity"
    elif rank == 0:
        out["cpu_baseline"] = None
    if rv is not None:
        rv.barrier()
    ctx.close()
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if rv is not None:
        rv.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
