#!/usr/bin/env python3
"""Summarise rocprofv3 runs of bench.py per hot-path TASK (the reference's operator):
average device time per task launch from the kernel trace, and HBM bytes per task launch
from separate FETCH_SIZE and WRITE_SIZE passes.  Writes the JSON that bench.py reads for
its roofline "traffic" (profiles/pmc_x1.<n>_L<L>.json, key "tasks").

A task is one or more kernels: its per-launch time is the summed kernel
time over the run divided by the number of task launches (launches per RK3 step x
steps, the steps counted from k_setup_cells, which runs exactly once per step).

Byte counters (MI355X_MICROARCH.md, HBM/rocprofv3): on gfx950 FETCH_SIZE tallies each
128-B L2->fabric read request as 64 B, so fetched bytes = 2 x FETCH_SIZE KiB x 1024;
Infinity-Cache hits are included (gather re-reads served on-die still count).  The
factor is checked on the pure-copy setup kernels, which fetch 4 whole 128-B lines per
column (levels 0..L-1 of the LP = 64 padded row).  WRITE_SIZE is calibrated the same
way against the setup kernels' written bytes (8 x L per column).

usage: pmc_summary.py --trace DIR --fetch DIR --write DIR --dims nC nE nV L --out FILE
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpas-regent_amd"))
from mpasdyn.pmc import read_trace, short, task_of  # noqa: E402,F401  (kernel -> task map shared with bench.py)

# task launches per RK3 step (schedule 1, x1.163842, the default fusions: setup + moist + stage
# 0's vert_imp in one launch, six dampings and the three set_smlstep inside acoustic launches,
# set_smlstep's flux sum once per step -- 7 acoustic substeps)
LAUNCHES = {"atm_rk_integration_setup": 1, "atm_compute_moist_coefficients": 1, "atm_compute_vert_imp_coefs": 1,
            "atm_compute_dyn_tend_work[rk0]": 1, "atm_compute_dyn_tend_work[rk>0]": 2,
            "atm_set_smlstep_pert_variables_work": 1, "atm_advance_acoustic_step_work": 7,
            "atm_divergence_damping_3d": 1, "atm_compute_solve_diagnostics": 3,
            "atm_rk_dynamics_substep_finish": 1}
# bench.py --physics / --transport (the MPAS vertical solver: 4 acoustic substeps and dampings,
# set_smlstep per stage, recover after every stage, the scalar transport once per step)
LAUNCHES_PHYSICS = dict(LAUNCHES, atm_advance_acoustic_step_work=4, atm_divergence_damping_3d=4,
                        atm_set_smlstep_pert_variables_work=3, atm_recover_large_step_variables_work=3,
                        atm_advance_scalars_mono=1)


def read_counter(d, counter):
    """total counter value and dispatch count per kernel over the run"""
    from mpasdyn.pmc import read_counter as rc
    r = rc(d, counter)
    return {k: v[0] for k, v in r.items()}, {k: v[1] for k, v in r.items()}


def once_per_step(d):
    """the step count of a run: the calls of a kernel that runs once per RK3 step (the separate
    setup copies of rounds 1-2, the fused setup launch since, or the substep finish)"""
    for k, v in d.items():
        if k in ("k_setup_cells", "k_copy64", "k_finish64") or k.startswith(("k_setup_vi<", "k_hf_setup_A<")):
            return v[0] if isinstance(v, tuple) else v
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--dims", nargs=4, type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--physics", action="store_true", help="the run was bench.py --physics or --transport")
    a = ap.parse_args()
    global LAUNCHES
    if a.physics:
        LAUNCHES = LAUNCHES_PHYSICS
    nC, nE, nV, L = a.dims
    out = {"dims": a.dims, "kernels": {}, "tasks": {}}
    tasks = defaultdict(lambda: {"kernels": [], "time_s": 0.0, "fetch_B": 0.0, "write_B": 0.0})
    steps = None
    if a.trace:
        tr = read_trace(a.trace)
        steps = once_per_step(tr)
        for k, (calls, t) in tr.items():
            out["kernels"][k] = {"calls": calls, "avg_us": round(t / calls * 1e6, 2)}
            task = task_of(k)
            if task and task in LAUNCHES:
                tasks[task]["kernels"].append(k)
                tasks[task]["time_s"] += t
    fetch, nf = read_counter(a.fetch, "FETCH_SIZE") if a.fetch else ({}, {})
    write, nw = read_counter(a.write, "WRITE_SIZE") if a.write else ({}, {})
    pmc_steps = once_per_step(nf) or once_per_step(nw)
    # calibration on the copies: setup_cells reads 6 cell fields and writes 7 (rho_zz
    # twice), setup_edges reads and writes 2 edge fields
    lines = {"k_setup_cells": 6 * nC * 4 * 128, "k_setup_edges": 2 * nE * 4 * 128, "k_copy64": (6 * nC + 2 * nE) * 4 * 128}
    payload = {"k_setup_cells": 7 * nC * 8 * L, "k_setup_edges": 2 * nE * 8 * L, "k_copy64": (7 * nC + 2 * nE) * 8 * L}
    ff = [lines[k] / (fetch[k] / nf[k] * 1024.0) for k in lines if fetch.get(k)]
    wf = [payload[k] / (write[k] / nw[k] * 1024.0) for k in payload if write.get(k)]
    out["fetch_factor_doc"] = 2.0
    out["fetch_factor_measured"] = round(sum(ff) / len(ff), 4) if ff else None
    out["write_factor_measured"] = round(sum(wf) / len(wf), 4) if wf else None
    wfac = out["write_factor_measured"] or 1.0
    for k in set(fetch) | set(write):
        d = out["kernels"].setdefault(k, {})
        if k in fetch:
            d["fetch_bytes_per_launch"] = 2.0 * fetch[k] / nf[k] * 1024.0
        if k in write:
            d["write_bytes_per_launch"] = wfac * write[k] / nw[k] * 1024.0
        task = task_of(k)
        if task and pmc_steps and task in LAUNCHES:
            tasks[task]["fetch_B"] += 2.0 * fetch.get(k, 0.0) * 1024.0
            tasks[task]["write_B"] += wfac * write.get(k, 0.0) * 1024.0
    for task, v in tasks.items():
        o = {"kernels": sorted(set(v["kernels"]))}
        if steps:
            o["avg_ms"] = round(v["time_s"] / (steps * LAUNCHES[task]) * 1e3, 4)
        if pmc_steps:
            n = pmc_steps * LAUNCHES[task]
            o["fetch_bytes_per_launch"] = v["fetch_B"] / n
            o["write_bytes_per_launch"] = v["write_B"] / n
            o["hbm_bytes_per_launch"] = (v["fetch_B"] + v["write_B"]) / n
        out["tasks"][task] = o
    out["steps_traced"], out["steps_counted"] = steps, pmc_steps
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1, sort_keys=True)
    for t, v in sorted(out["tasks"].items(), key=lambda kv: -kv[1].get("avg_ms", 0) * LAUNCHES[kv[0]]):
        print(f"{t:40s} avg_ms={v.get('avg_ms', 0):8.4f} x{LAUNCHES[t]}  "
              f"hbm_GB/launch={v.get('hbm_bytes_per_launch', 0) / 1e9:7.3f}")
    print("fetch factor measured", out["fetch_factor_measured"], "write factor", out["write_factor_measured"])


if __name__ == "__main__":
    main()
