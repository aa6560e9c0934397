#!/usr/bin/env python3
"""Traffic decomposition of atm_compute_dyn_tend_work: the HBM bytes its
kernels move per launch set, measured (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE, gfx950
correction of MI355X_MICROARCH.md), split into

    compulsory     the distinct arrays the whole task reads and writes, once each, at their
                   stored (LP-padded) size  -- the floor of any implementation in this layout
    intermediates  sum over kernels of each kernel's distinct arrays, minus the compulsory:
                   scratch written by one kernel and read back by another (X_F, X_wc), outputs
                   read back by a later kernel (kdiff, dpdz, delsq_*, tend_*_euler), inputs
                   read again by a later kernel -- the cost of the global barriers
    refetch        measured minus the per-kernel distinct bytes: columns fetched into an
                   XCD's L2 more than once (gathers whose neighbourhoods were evicted), partial
                   lines, the padding lanes

and B_alg (unpadded, the reference's read/write sets; mpasdyn/roofline.py).

usage: python tools/traffic_decomp.py KERNELS.txt [--dims 163842 491520 327680 56] [--lp 64]
       [--layout r03|r04] [--json OUT]
KERNELS.txt is tools/pmc_kernels.py output over FETCH_SIZE, WRITE_SIZE (and TCC) passes of one
bench step (tools/gpu.sh pmc).  --layout names the kernel sequence: r03 = A B C D E at rk_step 0
(D its own launch), r04 = option defer4 (no D; stage 1's B applies it)."""
import argparse
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mpas-regent_amd")]

# mesh rows a kernel loads, bytes per entity (the row_ld widths, not the stored widths)
MESH = {
    "A": ("C", 80 + 48 + 48 + 16 + 8 + 8 + 48 + 48),   # X_cR record, eocs, ce_dv, wfl, invArea, cosLat, defc_a/b (rk0)
    "B": ("E", 96 + 80 + 72 + 72 + 8 * 6),              # X_eB record, woe, adv_coefs(_3rd), scalars
    "C": ("C", 80 + 48 * 5),                            # + the vertex part below
    "Cv": ("V", 12 + 24 + 24 + 8),
    "D": ("E", 8 * 2 + 8 * 2 + 8 * 3),
    "E": ("C", 80 + 48 * 5 + 16),
}

# 3-D arrays per kernel (reads, writes) on the benchmark path: reference semantics, fast
# path (HF: B forms H per edge), fusecopy at stage 0.  kind by registry
KERN = {
    "r03": {
        "rk0": [
            ("A", ["ru", "u", "v", "rw", "rho_zz", "uReconstructZonal", "uReconstructMeridional", "tend_rho_physics",
                   "qtot", "rho_base", "rho_p_save"], ["kdiff", "h_divergence", "tend_rho", "dpdz", "X_wc"]),
            ("B", ["u", "ru", "rho_edge", "pv_edge", "tend_ru_physics", "cqu", "zxu", "rw", "w", "ke", "h_divergence",
                   "pressure_p", "zz", "dpdz", "divergence", "kdiff", "theta_m", "vorticity"],
             ["X_F", "tend_u", "tend_u_euler", "delsq_u", "ru_save", "u_2"]),
            ("C", ["delsq_u", "rho_edge", "kdiff", "X_wc", "theta_m"],
             ["delsq_vorticity", "delsq_divergence", "delsq_w", "tend_w_euler", "delsq_theta", "tend_theta_euler"]),
            ("D", ["rho_edge", "tend_u_euler", "tend_u", "tend_ru_physics", "delsq_divergence", "delsq_vorticity"],
             ["tend_u_euler", "tend_u"]),
            ("E", ["X_wc", "rw", "pressure_p", "dpdz", "rw_save", "theta_m_save", "theta_m", "tend_w_euler",
                   "tend_theta_euler", "rho_zz", "rt_diabatic_tend", "tend_rtheta_physics", "cqw", "delsq_w",
                   "delsq_theta", "X_F"],
             ["w", "tend_rtheta_adv", "rthdynten", "tend_theta", "tend_w_euler", "tend_theta_euler"]),
        ],
        "rk1": [
            ("A", ["ru", "rw", "rho_zz", "uReconstructZonal", "uReconstructMeridional"], ["h_divergence", "X_wc"]),
            ("B", ["u", "ru", "rho_edge", "pv_edge", "tend_ru_physics", "tend_u_euler", "ru_save", "rw", "w", "ke",
                   "h_divergence", "theta_m", "theta_m_save"], ["X_F", "tend_u"]),
            ("E", ["X_wc", "rw", "rw_save", "theta_m_save", "theta_m", "tend_w_euler", "tend_theta_euler", "rho_zz",
                   "rt_diabatic_tend", "tend_rtheta_physics", "X_F"],
             ["w", "tend_rtheta_adv", "rthdynten", "tend_theta"]),
        ],
    },
}
# option defer4 (r04): stage 0 runs A B C E (B stores no tend_u), stage 1's B applies D
_r04 = {"rk0": [k for k in KERN["r03"]["rk0"] if k[0] != "D"], "rk1": list(KERN["r03"]["rk1"])}
_r04["rk0"][1] = ("B", KERN["r03"]["rk0"][1][1], ["X_F", "tend_u_euler", "delsq_u", "ru_save", "u_2"])
_r04["rk1din"] = [k if k[0] != "B" else
                  ("B", k[1] + ["delsq_divergence", "delsq_vorticity"], k[2] + ["tend_u_euler"])
                  for k in KERN["r03"]["rk1"]]
# (the plain rk_step > 0 launch is stage 2's, whose B also stores v: option vdyn; E forms wc)
_r04["rk1"] = [("A", ["ru"], ["h_divergence"]) if k[0] == "A" else
               ("B", k[1], k[2] + ["v"]) if k[0] == "B" else
               ("E", [f for f in k[1] if f != "X_wc"] + ["ru", "uReconstructZonal", "uReconstructMeridional"], k[2])
               for k in KERN["r03"]["rk1"]]
_r04["rk1din"] = [("A", ["ru"], ["h_divergence"]) if k[0] == "A" else
                  ("E", [f for f in k[1] if f != "X_wc"] + ["ru", "uReconstructZonal", "uReconstructMeridional"], k[2])
                  if k[0] == "E" else k for k in _r04["rk1din"]]
KERN["r04"] = _r04

# the kernel names of the rocprofv3 output per launch kind
PAT = {
    ("rk0", "A"): r"^k_dyn_A<64, true", ("rk0", "B"): r"^k_dyn_B<64, true", ("rk0", "C"): r"^k_dyn_C(12)?<64",
    ("rk0", "D"): r"^k_dyn_D<64", ("rk0", "E"): r"^k_dyn_E<64, true",
    ("rk1", "A"): r"^k_dyn_A<64, false", ("rk1", "B"): r"^k_dyn_B<64, false, false, true(, false)?>$",
    ("rk1", "E"): r"^k_dyn_E<64, false",
    ("rk1din", "A"): r"^k_dyn_A<64, false", ("rk1din", "B"): r"^k_dyn_B<64, false, false, true, true>",
    ("rk1din", "E"): r"^k_dyn_E<64, false",
}


def field_kind(name):
    from mpasdyn import registry
    if name.startswith("X_"):
        return {"X_wc": "C", "X_F": "E"}[name]
    return registry.BY_NAME[name].kind[0]


def parse_kernels(path):
    out, cur = {}, None
    for line in open(path):
        if not line.startswith(" "):
            cur = line.strip()
            out[cur] = {}
        else:
            k, v = line.split()
            out[cur][k] = float(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("--dims", type=int, nargs=4, default=[163842, 491520, 327680, 56])
    ap.add_argument("--lp", type=int, default=64)
    ap.add_argument("--layout", default="r03")
    ap.add_argument("--json")
    a = ap.parse_args()
    nC, nE, nV, L = a.dims
    n = {"C": nC, "E": nE, "V": nV}
    col = lambda kind: 8.0 * n[kind] * a.lp  # noqa: E731
    pmc = parse_kernels(a.kernels)
    from mpasdyn import roofline

    res = {}
    kinds = ["rk0", "rk1"] + (["rk1din"] if a.layout == "r04" else [])
    for lk in kinds:
        kern = KERN[a.layout][lk]
        per, tot_kernel, meas_tot = [], 0.0, 0.0
        task_r, task_w = set(), set()
        for name, rd, wr in kern:
            kind_mesh = MESH[name]
            comp = sum(col(field_kind(f)) for f in set(rd)) + sum(col(field_kind(f)) for f in set(wr))
            comp += kind_mesh[1] * n[kind_mesh[0]]
            if name == "C":
                comp += MESH["Cv"][1] * nV
            task_r |= set(f for f in rd if f not in task_w)
            task_w |= set(wr)
            m = [v for kname, v in pmc.items() if re.search(PAT[(lk, name)], kname)]
            # (every matching kernel summed: C is two launches, its vertex and its cell blocks)
            if not m:
                meas = None
            else:
                meas = 1e3 * sum(2 * x["FETCH_SIZE"] + x["WRITE_SIZE"] for x in m)  # KB -> B; FETCH x 2 (gfx950)
            hit = None
            if m and all("TCC_HIT_sum" in x for x in m):
                h = sum(x["TCC_HIT_sum"] for x in m)
                hit = h / (h + sum(x["TCC_MISS_sum"] for x in m))
            per.append({"kernel": name, "compulsory_GB": comp / 1e9, "measured_GB": None if meas is None else meas / 1e9,
                        "refetch_GB": None if meas is None else (meas - comp) / 1e9, "l2_hit": hit})
            tot_kernel += comp
            meas_tot += meas or 0.0
        scratch = {"X_wc", "X_F"}
        task = sum(col(field_kind(f)) for f in task_r - scratch) + sum(col(field_kind(f)) for f in task_w - scratch)
        task += sum(MESH[k[0]][1] * n[MESH[k[0]][0]] for k in kern)  # (mesh rows once per kernel: a floor)
        balg = roofline.b_alg("atm_compute_dyn_tend_work", (nC, nE, nV, L), rk_step=0 if lk == "rk0" else 1,
                              copy=(lk == "rk0"))
        res[lk] = {"kernels": per, "B_alg_GB": balg / 1e9, "compulsory_GB": task / 1e9,
                   "intermediates_GB": (tot_kernel - task) / 1e9, "refetch_GB": (meas_tot - tot_kernel) / 1e9,
                   "measured_GB": meas_tot / 1e9, "measured_over_B_alg": meas_tot / balg}
    # per array: which kernel writes it, which read it, and the bytes it
    # moves beyond its compulsory once -- each kernel touching it moves its stored size (the
    # distinct bytes, no refetch); a scratch array (X_*) has no compulsory part
    arrays = {}
    for lk in kinds:
        rows = {}
        for name, rd, wr in KERN[a.layout][lk]:
            for f in dict.fromkeys(rd + wr):
                r = rows.setdefault(f, {"writers": [], "readers": [], "GB": col(field_kind(f)) / 1e9})
                if f in wr:
                    r["writers"].append(name)
                if f in rd:
                    r["readers"].append(name)
        for f, r in rows.items():
            touches = len(set(r["writers"]) | set(r["readers"])) + sum(
                1 for w in set(r["writers"]) if w in r["readers"])  # (read and written by one kernel: twice)
            r["extra_GB"] = r["GB"] * (touches - (0 if f.startswith("X_") else 1))
        arrays[lk] = dict(sorted(((f, r) for f, r in rows.items() if r["extra_GB"] > 0),
                                 key=lambda x: -x[1]["extra_GB"]))
        res[lk]["arrays"] = arrays[lk]
    print(f"dyn_tend traffic decomposition ({a.layout}), x1.{nC} x {L}, LP {a.lp}, GB per launch")
    for lk, d in res.items():
        print(f"{lk:7s} measured {d['measured_GB']:6.2f} = compulsory {d['compulsory_GB']:5.2f} + intermediates "
              f"{d['intermediates_GB']:5.2f} + refetch {d['refetch_GB']:5.2f};  B_alg {d['B_alg_GB']:5.2f}, "
              f"measured / B_alg {d['measured_over_B_alg']:4.2f}")
        for k in d["kernels"]:
            ms = "--" if k["measured_GB"] is None else f"{k['measured_GB']:5.2f}"
            rf = "--" if k["refetch_GB"] is None else f"{k['refetch_GB']:5.2f}"
            l2 = "--" if k["l2_hit"] is None else f"{k['l2_hit']:.2f}"
            print(f"    {k['kernel']}: measured {ms}  distinct {k['compulsory_GB']:5.2f}  refetch {rf}  L2 hit {l2}")
    for lk, rows in arrays.items():
        print(f"{lk}: arrays moved more than once (extra GB per launch beyond the compulsory once)")
        for f, r in rows.items():
            print(f"    {f:22s} {r['extra_GB']:5.3f}  written by {','.join(r['writers']) or '-':6s} "
                  f"read by {','.join(r['readers'])}")
        print(f"    sum {sum(r['extra_GB'] for r in rows.values()):.2f}")
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
