#!/usr/bin/env python3
"""Traffic decomposition of atm_compute_dyn_tend_work: the HBM
bytes its kernels move per launch, measured (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE, the gfx950
correction of MI355X_MICROARCH.md), split into

    compulsory     the distinct arrays the whole task reads and writes, once each, at their
                   stored (LP-padded) size -- the floor of any implementation in this layout
    intermediates  sum over kernels of each kernel's distinct arrays, minus the compulsory:
                   scratch written by one kernel and read back by another (X_F, X_wc), outputs
                   read back by a later kernel (kdiff, dpdz, delsq_*, tend_*_euler), inputs
                   read again by a later kernel -- the cost of the global barriers
    refetch        measured minus the per-kernel distinct bytes: columns fetched into an
                   XCD's L2 more than once (gathers whose neighbourhoods were evicted), partial
                   lines, the padding lanes

and B_alg (unpadded, the reference's read/write sets; mpasdyn/roofline.py).

usage: python tools/traffic_decomp.py KERNELS.txt --layout r05|r06|r06ntu [--round r06]
       [--dims 163842 491520 327680 56] [--lp 64] [--json OUT]
KERNELS.txt is tools/pmc_kernels.py output over the FETCH_SIZE and WRITE_SIZE (and TCC) passes of
one bench step (tools/gpu.sh pmc).  Layouts (the kernels of the benchmark path, every variant by its
template arguments):
    r05  round 5's path: A, B (fast path: B forms each edge's theta flux H into X_F), C, E; rk_step 0
         leaves D to stage 1's B (defer4: B's DIN variant), stage 2's B stores v (vdyn)
    r06  option etile: B forms no flux (its NOF variant), the tiled E (k_dyn_Et) forms each edge's flux
         from its tile's theta_m columns in LDS; no X_F
    r06ntu  option ntu (round 6's default path): stage 0's B forms no tend_u and no flux, its E no theta
         tendency; stage 1 is E's w alone; stage 2's B applies the deferred del4 and stores v
The tool fails (exit status 2) when a dyn_tend kernel of the file matches no kernel of the layout,
when a kernel of the layout is missing from the file, or when a kernel's measured bytes fall below
its distinct bytes (a negative refetch: the layout's read / write set of that kernel is wrong)."""
import argparse
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mpas-regent_amd")]

# A kernel name as pmc_kernels.py prints it, e.g. "k_dyn_B<64, false, false, true, true, false>":
# the template arguments in order (bools as 0/1, ints as ints)
def targs(name):
    m = re.match(r"^(k_dyn_\w+)<([^>]*)>$", name.strip())
    if not m:
        return None, None
    args = []
    for a in m.group(2).split(","):
        a = a.strip()
        args.append(1 if a == "true" else 0 if a == "false" else int(a))
    return m.group(1), tuple(args)


# Each kernel of a layout: (label, kernel, predicate over its template arguments, reads, writes, mesh)
#   reads / writes: 3-D arrays; "f:C" = only nCells columns of the (edge) array f are touched
#   mesh: (entity kind, bytes per entity) of the mesh rows and tables the kernel loads
B_RK0_R = ["u", "ru", "rho_edge", "pv_edge", "tend_ru_physics", "cqu", "zxu", "rw", "w", "ke", "h_divergence",
           "pressure_p", "zz", "dpdz", "divergence", "kdiff", "vorticity"]
B_RK1_R = ["u", "ru", "rho_edge", "pv_edge", "tend_ru_physics", "tend_u_euler", "rw", "w", "ke", "h_divergence"]
E_RK1_R = ["rw", "rw_save", "theta_m_save", "theta_m", "tend_w_euler", "tend_theta_euler", "rho_zz",
           "rt_diabatic_tend", "tend_rtheta_physics", "uReconstructZonal", "uReconstructMeridional"]
E_RK0_R = ["X_wc", "rw", "pressure_p", "dpdz", "rw_save", "theta_m_save", "theta_m", "tend_w_euler",
           "tend_theta_euler", "rho_zz", "rt_diabatic_tend", "tend_rtheta_physics", "cqw", "delsq_w", "delsq_theta"]
E_W = ["w", "tend_rtheta_adv", "rthdynten", "tend_theta"]
E_EB = 96 + 4 + 8 + 8 * 6  # X_eB record, nEdgesOnEdge...: B's index record and per-edge scalars
W_EDGE = 80                 # weightsOnEdge row (QF doubles)
ADV_EDGE = 72 + 72          # adv_coefs, adv_coefs_3rd (AF doubles each)
C_REC = 80 + 48 + 48         # X_cR record, edgesOnCell_sign, ce_dv
A_KS = [
    ("A", "k_dyn_A", lambda t: t[1] == 1, ["ru", "u", "v", "rw", "rho_zz", "uReconstructZonal",
                                            "uReconstructMeridional", "tend_rho_physics", "qtot", "rho_base",
                                            "rho_p_save"], ["kdiff", "h_divergence", "tend_rho", "dpdz", "X_wc"],
     ("C", C_REC + 16 + 8 + 8 + 48 + 48)),
]
A_K1 = ("A", "k_dyn_A", lambda t: t[1] == 0, ["ru"], ["h_divergence"], ("C", C_REC + 8))
C_K = ("C", "k_dyn_C12", lambda t: True, ["delsq_u", "rho_edge", "kdiff", "X_wc", "theta_m"],
       ["delsq_vorticity", "delsq_divergence", "delsq_w", "tend_w_euler", "delsq_theta", "tend_theta_euler"],
       ("C", C_REC + 48 * 3 + 12 * 0))
LAYOUTS = {
    "r05": {
        "rk0": A_KS + [
            ("B", "k_dyn_B", lambda t: t[1:] == (1, 0, 1, 0, 0), B_RK0_R + ["theta_m"],
             ["X_F", "tend_u_euler", "delsq_u", "ru_save", "u_2"], ("E", E_EB + W_EDGE + ADV_EDGE)),
            C_K,
            ("E", "k_dyn_E", lambda t: t[1] == 1 and t[3:] == (0, 1), E_RK0_R + ["X_F"], E_W + ["tend_w_euler",
                                                                                           "tend_theta_euler"],
             ("C", C_REC + 48 * 2 + 8)),
        ],
        "rk1din": [
            A_K1,
            ("B", "k_dyn_B", lambda t: t[1:] == (0, 0, 1, 1, 0),
             B_RK1_R + ["theta_m", "ru_save", "theta_m_save", "delsq_divergence", "delsq_vorticity"],
             ["X_F", "tend_u", "tend_u_euler"], ("E", E_EB + W_EDGE + ADV_EDGE)),
            ("E", "k_dyn_E", lambda t: t[1] == 0 and t[3:] == (0, 1), E_RK1_R + ["ru:C", "X_F"], E_W,
             ("C", C_REC + 16 + 8 + 8)),
        ],
        "rk1": [
            A_K1,
            ("B", "k_dyn_B", lambda t: t[1:] == (0, 0, 1, 0, 0), B_RK1_R + ["theta_m", "ru_save", "theta_m_save"],
             ["X_F", "tend_u", "v"], ("E", E_EB + W_EDGE + ADV_EDGE)),
            ("E", "k_dyn_E", lambda t: t[1] == 0 and t[3:] == (0, 1), E_RK1_R + ["ru:C", "X_F"], E_W,
             ("C", C_REC + 16 + 8 + 8)),
        ],
    },
}
# r06 (option etile): B without the flux (NOF), the tiled E (k_dyn_Et<RK0, SELF, HF>) reads ru at every
# edge of its cells, ru_save / theta_m_save at rk_step > 0 and the tile's theta_m closure; mesh: its
# cell records (72 B), the tiles' edge lists and the edges' adv_coefs / adv_coefs_3rd rows
ET_MESH_C = C_REC + 72 + 8 + 8
_r06 = {"rk0": [], "rk1din": [], "rk1": []}
for lk, ks in LAYOUTS["r05"].items():
    for k in ks:
        if k[0] == "B":
            rd = [f for f in k[3] if f not in ("theta_m", "ru_save", "theta_m_save")]
            wr = [f for f in k[4] if f != "X_F"]
            pred = {"rk0": lambda t: t[1:] == (1, 0, 1, 0, 1), "rk1din": lambda t: t[1:] == (0, 0, 1, 1, 1),
                    "rk1": lambda t: t[1:] == (0, 0, 1, 0, 1)}[lk]
            _r06[lk].append(("B", "k_dyn_B", pred, rd, wr, ("E", E_EB + W_EDGE)))
        elif k[0] == "E":
            rd = [f for f in k[3] if f not in ("X_F", "ru:C")] + ["ru"] + ([] if lk == "rk0" else [])
            pred = (lambda t: t[0] == 1 and t[2] == 1) if lk == "rk0" else (lambda t: t[0] == 0 and t[2] == 1)
            _r06[lk].append(("E", "k_dyn_Et", pred, rd, k[4], ("C", ET_MESH_C, "E", ADV_EDGE + 8)))
        else:
            _r06[lk].append(k)
LAYOUTS["r06"] = _r06
# r06ntu (option ntu, the round-6 default path; k_dyn_B<LP, RK0, MD, HF, DIN, NOF, NTU>,
# k_dyn_E<LP, RK0, SELF, MD, HF, NTH>): stage 0 (rk_step 0) -- B forms no tend_u and no flux (NOF, NTU:
# the pressure gradient, del2 and setup's copies), E no theta tendency (NTH: w, tend_w_euler and
# tend_theta_euler with their del4); stage 1 (rk_step > 0) -- E's w alone; stage 2 -- A, B with the
# deferred del4 (DIN) and v (vdyn), E
B_RK0_NTU_R = ["u", "ru", "rho_edge", "cqu", "zxu", "pressure_p", "zz", "dpdz", "divergence", "kdiff", "vorticity"]
E_RK0_NTH_R = ["X_wc", "rw", "pressure_p", "dpdz", "theta_m", "tend_w_euler", "tend_theta_euler", "rho_zz", "cqw",
               "delsq_w", "delsq_theta"]
E_RK1_NTH_R = ["uReconstructZonal", "uReconstructMeridional", "rw", "ru:C", "theta_m", "tend_w_euler",
               "tend_theta_euler", "rho_zz"]
# (A at rk_step 0 stores no h_divergence: B forms no tend_u, its only reader)
A_KS_NTU = [(k[0], k[1], k[2], k[3], [f for f in k[4] if f != "h_divergence"], k[5]) for k in A_KS]
LAYOUTS["r06ntu"] = {
    "rk0": A_KS_NTU + [
        ("B", "k_dyn_B", lambda t: t[1:] == (1, 0, 1, 0, 1, 1), B_RK0_NTU_R,
         ["tend_u_euler", "delsq_u", "ru_save", "u_2"], ("E", E_EB)),
        C_K,
        ("E", "k_dyn_E", lambda t: t[1] == 1 and t[3:] == (0, 1, 1), E_RK0_NTH_R,
         ["w", "tend_w_euler", "tend_theta_euler"], ("C", C_REC + 48 * 2 + 8)),
    ],
    "rk1ntu": [
        ("E", "k_dyn_E", lambda t: t[1] == 0 and t[3:] == (0, 1, 1), E_RK1_NTH_R, ["w"], ("C", C_REC + 16 + 8 + 8)),
    ],
    "rk1dinv": [
        A_K1,
        ("B", "k_dyn_B", lambda t: t[1:] == (0, 0, 1, 1, 0, 0),
         B_RK1_R + ["theta_m", "ru_save", "theta_m_save", "delsq_divergence", "delsq_vorticity"],
         ["X_F", "tend_u", "tend_u_euler", "v"], ("E", E_EB + W_EDGE + ADV_EDGE)),
        ("E", "k_dyn_E", lambda t: t[1] == 0 and t[3:] == (0, 1, 0), E_RK1_R + ["ru:C", "X_F"], E_W,
         ("C", C_REC + 16 + 8 + 8)),
    ],
}
# B_alg of each launch kind (mpasdyn/roofline.py); default: rk_step and stage 0's copies
BALG_KW = {"r06ntu": {"rk0": {"rk_step": 0, "copy": True, "defer_out": True, "ntu": True},
                      "rk1ntu": {"rk_step": 1, "ntu": True}, "rk1dinv": {"rk_step": 1, "store_v": True}}}
SCRATCH = {"X_wc", "X_F"}


def field_kind(name):
    from mpasdyn import registry
    if name.startswith("X_"):
        return {"X_wc": "C", "X_F": "E"}[name]
    return registry.BY_NAME[name].kind[0]


def parse_kernels(path):
    out, cur = {}, None
    for line in open(path):
        if not line.strip():
            continue
        if not line.startswith(" "):
            cur = line.strip()
            out[cur] = {}
        else:
            k, v = line.split()
            out[cur][k] = float(v)
    return out


class DecompError(Exception):
    pass


def decompose(pmc, layout, dims, lp=64):
    """the decomposition of every launch kind of `layout` from the per-kernel counters `pmc`
    ({kernel name: {counter: mean value}}, FETCH_SIZE / WRITE_SIZE in KB); raises DecompError on an
    unmatched or missing kernel and on a negative refetch"""
    from mpasdyn import roofline
    nC, nE, nV, L = dims
    n = {"C": nC, "E": nE, "V": nV}
    lay = LAYOUTS[layout]

    def col(f):
        if f.endswith(":C"):
            return 8.0 * nC * lp
        return 8.0 * n[field_kind(f)] * lp

    def fname(f):
        return f.split(":")[0]

    # every dyn_tend kernel of the file is claimed by exactly the kernels of the layout
    claimed = {}
    for name in pmc:
        kern, t = targs(name)
        if kern is None or not kern.startswith("k_dyn"):
            continue
        hits = [(lk, k[0]) for lk, ks in lay.items() for k in ks if k[1] == kern and k[2](t)]
        if not hits:
            raise DecompError(f"kernel {name} matches no kernel of layout {layout}")
        claimed[name] = hits
    res = {}
    for lk, ks in lay.items():
        per, tot_kernel, meas_tot = [], 0.0, 0.0
        task_r, task_w = {}, set()  # (task_r: array -> its bytes; "f:C" counts nCells columns unless read whole)
        for label, kern, pred, rd, wr, mesh in ks:
            m = [v for name, v in pmc.items() if (lk, label) in claimed.get(name, ())]
            if not m:
                raise DecompError(f"{lk} {label}: no {kern} kernel of layout {layout} in the counters")
            comp = sum(col(f) for f in set(rd)) + sum(col(f) for f in set(wr))
            for q in range(0, len(mesh), 2):
                comp += mesh[q + 1] * n[mesh[q]]
            if label == "C":
                comp += (12 + 24 + 24 + 8) * nV  # the vertex blocks' rows
            for f in rd:
                if fname(f) not in task_w:
                    task_r[fname(f)] = max(task_r.get(fname(f), 0.0), col(f))
            task_w |= set(wr)
            meas = 1e3 * sum(2 * x["FETCH_SIZE"] + x["WRITE_SIZE"] for x in m)  # KB -> B; FETCH x 2 (gfx950)
            hit = None
            if all("TCC_HIT_sum" in x for x in m):
                h = sum(x["TCC_HIT_sum"] for x in m)
                hit = h / max(h + sum(x["TCC_MISS_sum"] for x in m), 1.0)
            if meas < comp:
                raise DecompError(f"{lk} {label}: measured {meas / 1e9:.3f} GB below its distinct {comp / 1e9:.3f} GB "
                                  f"(negative refetch: the layout's read / write set is wrong)")
            per.append({"kernel": label, "names": sorted(nm for nm in claimed if (lk, label) in claimed[nm]),
                        "compulsory_GB": comp / 1e9, "measured_GB": meas / 1e9, "refetch_GB": (meas - comp) / 1e9,
                        "l2_hit": hit})
            tot_kernel += comp
            meas_tot += meas
        task = sum(b for f, b in task_r.items() if f not in SCRATCH) + sum(col(f) for f in task_w - SCRATCH)
        for k in ks:  # (mesh rows once per kernel: a floor)
            for q in range(0, len(k[5]), 2):
                task += k[5][q + 1] * n[k[5][q]]
        kw = BALG_KW.get(layout, {}).get(lk, {"rk_step": 0 if lk == "rk0" else 1, "copy": lk == "rk0"})
        balg = roofline.b_alg("atm_compute_dyn_tend_work", (nC, nE, nV, L), **kw)
        res[lk] = {"kernels": per, "B_alg_GB": balg / 1e9, "compulsory_GB": task / 1e9,
                   "intermediates_GB": (tot_kernel - task) / 1e9, "refetch_GB": (meas_tot - tot_kernel) / 1e9,
                   "measured_GB": meas_tot / 1e9, "measured_over_B_alg": meas_tot / balg}
        # per array: which kernel writes it, which read it, and the bytes it moves beyond its
        # compulsory once (a scratch array X_* has no compulsory part)
        rows = {}
        for label, _, _, rd, wr, _ in ks:
            for f in dict.fromkeys(rd + wr):
                r = rows.setdefault(fname(f), {"writers": [], "readers": [], "GB": col(fname(f)) / 1e9})
                if f in wr:
                    r["writers"].append(label)
                if f in rd:
                    r["readers"].append(label)
        for f, r in rows.items():
            touches = len(set(r["writers"]) | set(r["readers"])) + sum(1 for w in set(r["writers"]) if w in r["readers"])
            r["extra_GB"] = r["GB"] * (touches - (0 if f.startswith("X_") else 1))
        res[lk]["arrays"] = dict(sorted(((f, r) for f, r in rows.items() if r["extra_GB"] > 0),
                                        key=lambda x: -x[1]["extra_GB"]))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("--dims", type=int, nargs=4, default=[163842, 491520, 327680, 56])
    ap.add_argument("--lp", type=int, default=64)
    ap.add_argument("--layout", required=True, choices=sorted(LAYOUTS))
    ap.add_argument("--round", default="", help="the round the counters were taken in (the header's label)")
    ap.add_argument("--json")
    a = ap.parse_args()
    nC, nE, nV, L = a.dims
    try:
        res = decompose(parse_kernels(a.kernels), a.layout, a.dims, a.lp)
    except DecompError as e:
        print(f"traffic_decomp: {e}", file=sys.stderr)
        return 2
    rnd = f" {a.round}" if a.round else ""
    print(f"dyn_tend traffic decomposition{rnd} (layout {a.layout}), x1.{nC} x {L}, LP {a.lp}, GB per launch")
    for lk, d in res.items():
        print(f"{lk:7s} measured {d['measured_GB']:6.2f} = compulsory {d['compulsory_GB']:5.2f} + intermediates "
              f"{d['intermediates_GB']:5.2f} + refetch {d['refetch_GB']:5.2f};  B_alg {d['B_alg_GB']:5.2f}, "
              f"measured / B_alg {d['measured_over_B_alg']:4.2f}")
        for k in d["kernels"]:
            l2 = "--" if k["l2_hit"] is None else f"{k['l2_hit']:.2f}"
            print(f"    {k['kernel']}: measured {k['measured_GB']:5.2f}  distinct {k['compulsory_GB']:5.2f}  "
                  f"refetch {k['refetch_GB']:5.2f}  L2 hit {l2}  ({'; '.join(k['names'])})")
    for lk, d in res.items():
        print(f"{lk}: arrays moved more than once (extra GB per launch beyond the compulsory once)")
        for f, r in d["arrays"].items():
            print(f"    {f:22s} {r['extra_GB']:5.3f}  written by {','.join(r['writers']) or '-':6s} "
                  f"read by {','.join(r['readers'])}")
        print(f"    sum {sum(r['extra_GB'] for r in d['arrays'].values()):.2f}")
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
