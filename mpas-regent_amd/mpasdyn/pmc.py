"""Reading rocprofv3 output per hot-path TASK (the reference's operator).

A task is one or more kernels.  HBM bytes come from separate FETCH_SIZE
and WRITE_SIZE passes (MI355X_MICROARCH.md, HBM/rocprofv3: the two cannot share a pass;
on gfx950 FETCH_SIZE tallies each 128-B L2->fabric read request as 64 B, so fetched
bytes = 2 x FETCH_SIZE KiB x 1024; Infinity-Cache hits are included).  WRITE_SIZE is
calibrated on the pure-copy setup kernels (the same check the fetch factor gets).

Used by bench.py (live traffic of the timed workload) and tools/pmc_summary.py.
"""
import csv
import glob
import os
import re
from collections import defaultdict

# kernel -> timing key of the task it belongs to (first regex that matches)
KERNEL_TASK = [
    # (option fusesetup: setup + moist + stage 0's vert_imp in one launch, timed as setup)
    (r"k_setup_(cells|edges|vi)|k_copy64", "atm_rk_integration_setup"),
    (r"k_moist", "atm_compute_moist_coefficients"),
    (r"k_vert_imp", "atm_compute_vert_imp_coefs"),
    (r"k_dyn_(Bf|[ABE])<\d+, true", "atm_compute_dyn_tend_work[rk0]"),
    (r"k_dyn_([CD]|DE|C12)<", "atm_compute_dyn_tend_work[rk0]"),
    # option hfuse: launches shared by two tasks (timing keys hfuse[a+b])
    (r"k_hf_", "hfuse"),
    (r"k_dyn_(Bf|[ABE])<\d+, false", "atm_compute_dyn_tend_work[rk>0]"),
    (r"k_set_smlstep|k_sml_flux", "atm_set_smlstep_pert_variables_work"),
    (r"k_acoustic", "atm_advance_acoustic_step_work"),
    (r"k_div_damp", "atm_divergence_damping_3d"),
    (r"k_solve_", "atm_compute_solve_diagnostics"),
    (r"k_finish_|k_finish64", "atm_rk_dynamics_substep_finish"),
    (r"k_recover_", "atm_recover_large_step_variables_work"),
    (r"k_tr_", "atm_advance_scalars_mono"),
]
FETCH_FACTOR = 2.0  # MI355X_MICROARCH.md: gfx950 FETCH_SIZE is half the fetched bytes


def task_of(kernel):
    for pat, task in KERNEL_TASK:
        if re.search(pat, kernel):
            return task
    return None


def short(name):
    return name.replace("void ", "").replace("mpas::", "").split("(")[0]


def read_counter(d, counter):
    """{kernel: (summed counter value, dispatches)} of a rocprofv3 --pmc output dir"""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise FileNotFoundError(f"no counter_collection.csv under {d}")
    tot, n = defaultdict(float), defaultdict(int)
    for f in files:
        with open(f) as fo:
            for r in csv.DictReader(fo):
                if r["Counter_Name"] == counter:
                    k = short(r["Kernel_Name"])
                    tot[k] += float(r["Counter_Value"])
                    n[k] += 1
    return {k: (tot[k], n[k]) for k in tot}


def read_trace(d):
    """{kernel: (calls, total seconds)} of a rocprofv3 --kernel-trace --stats output dir"""
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    out = {}
    with open(f) as fo:
        for r in csv.DictReader(fo):
            out[short(r["Name"])] = (int(r["Calls"]), float(r["TotalDurationNs"]) * 1e-9)
    return out


def write_factor(write, nCells, nEdges, L, physics=0):
    """WRITE_SIZE KiB -> bytes factor, measured on the copy kernels of the setup task
    (setup_cells writes 7 cell fields -- 8 under the MPAS dynamics, which also saves
    theta_m --, setup_edges 2 edge fields, levels 0..L-1; at LP 64 one k_copy64 launch
    writes both)"""
    nc = 8 if physics == 2 else 7
    payload = {"k_setup_cells": nc * nCells * 8 * L, "k_setup_edges": 2 * nEdges * 8 * L,
               "k_copy64": (nc * nCells + 2 * nEdges) * 8 * L}
    f = [payload[k] / (write[k][0] / write[k][1] * 1024.0) for k in payload if k in write and write[k][0] > 0]
    return sum(f) / len(f) if f else None


CALIBRATION_KERNELS = ("k_copy64", "k_setup_cells", "k_setup_edges")


def drop_calibration(counts):
    """remove one dispatch (the last, a standalone atm_rk_integration_setup run after the
    counted step so that the copy kernels exist whatever the step fuses) from each
    calibration kernel's {kernel: (value, dispatches)} entry"""
    out = dict(counts)
    for k in CALIBRATION_KERNELS:
        if k in out:
            v, n = out[k]
            if n > 1:
                out[k] = (v * (n - 1) / n, n - 1)
            else:
                del out[k]
    return out


def bytes_per_step(fetch, write, steps, wfac):
    """{timing key: (fetched bytes, written bytes) per RK3 step} over the dispatches of
    the counted run (`steps` whole RK3 steps)"""
    out = defaultdict(lambda: [0.0, 0.0])
    for k, (v, _) in fetch.items():
        t = task_of(k)
        if t:
            out[t][0] += FETCH_FACTOR * v * 1024.0 / steps
    for k, (v, _) in write.items():
        t = task_of(k)
        if t:
            out[t][1] += wfac * v * 1024.0 / steps
    return {t: tuple(v) for t, v in out.items()}
