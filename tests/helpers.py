"""Shared test helpers: state construction through the oracle's generator, and the
comparison rule used for GPU-vs-oracle parity."""
import numpy as np

from mpasdyn import build_state as bs
from mpasdyn.registry import FIELDS

# fields the reference uses as per-task scratch (kept in registers on the GPU; their
# values after a task are not part of the result, SURVEY §8.5 B_alg note)
SCRATCH = {"flux_arr", "ru_edge_w", "wduz", "q", "wdwz", "wdtz", "u_mix"}

SEED = 20211015


def make_state(mesh, L, variant, seed=SEED):
    import oracle as O
    fill = lambda st, s, inc: O.Oracle(st).fill_synthetic(s, inc)  # noqa: E731
    return bs.build_state(mesh, L, variant, seed=seed, oracle_fill=fill)


# fields whose zero slot (row n, the Q1 garbage entity) a task of the path writes: the
# recover step's "garbage cell" rho_zz (dynamics_tasks.rg:1766-1872 reads and writes the
# cell that raw id n resolves to, Q7 path).  Downloads cover the n entities only, so the
# device's row n is not observable and is excluded by rule; the entities that read it
# (u at every edge whose raw cellsOnEdge is n) carry its value into the comparison.
ZERO_SLOT_WRITTEN = ("rho_zz",)


def compare_states(got, ref, rtol=0.0, fields=None, skip=SCRATCH, tol_fields=None, zero_slot_excluded=()):
    """Return a list of (field, max_abs_err, scale) mismatches.

    rtol == 0 demands bit-identical arrays (NaNs must sit at the same places).
    Otherwise |got - ref| <= rtol * max|ref| per field (normwise), for the fields in
    tol_fields (all fields when tol_fields is None); the others stay bit-exact.
    zero_slot_excluded: fields compared on rows [0, n) only (ZERO_SLOT_WRITTEN)."""
    bad = []
    for f in FIELDS:
        if f.name in skip or (fields is not None and f.name not in fields):
            continue
        a, b = got.arrays[f.name], ref.arrays[f.name]
        if f.name in zero_slot_excluded:
            n = got.n_of(f)
            a, b = a[:n], b[:n]
        tol = rtol if (tol_fields is None or f.name in tol_fields) else 0.0
        if f.dtype != np.float64:
            if not np.array_equal(a, b):
                bad.append((f.name, "int mismatch", None))
            continue
        na, nb = np.isnan(a), np.isnan(b)
        if not np.array_equal(na, nb):
            bad.append((f.name, f"nan mask differs ({na.sum()} vs {nb.sum()})", None))
            continue
        a2, b2 = np.where(na, 0.0, a), np.where(nb, 0.0, b)
        if tol == 0.0:
            if not np.array_equal(a2, b2):  # value-identical (+0 == -0)
                with np.errstate(invalid="ignore"):
                    d = np.abs(a2 - b2)
                bad.append((f.name, float(np.nanmax(d)), float(np.nanmax(np.abs(b2)))))
        else:
            fin = np.isfinite(b2)
            scale = float(np.max(np.abs(b2[fin]))) if fin.any() else 0.0
            d = np.abs(a2 - b2)[fin]
            err = float(d.max()) if d.size else 0.0
            if err > rtol * max(scale, 1e-300) or not np.array_equal(np.isinf(a2), np.isinf(b2)):
                bad.append((f.name, err, scale))
    return bad


def digest(a):
    """order-sensitive fingerprint of an array for the golden fixtures"""
    import hashlib
    a = np.ascontiguousarray(a)
    if a.dtype == np.float64:
        r = np.where(np.isfinite(a), a, 0.0)
        return {"sum": float(np.sum(r)), "l2": float(np.sqrt(np.sum(r * r))), "min": float(np.min(r)),
                "max": float(np.max(r)), "sha": hashlib.sha256(a.tobytes()).hexdigest()[:32]}
    return {"sum": int(np.sum(a, dtype=np.int64)), "sha": hashlib.sha256(a.tobytes()).hexdigest()[:32]}


def transport_state(mesh, L, dt, seed=SEED, const=None):
    """A state for the monotonic scalar transport (Q26; mpas mode): the real x1 geometry in
    0-based ids ("physical" variant), a smooth rotating flow plus noise in ruAvg, a
    random vertical mass flux wwAvg (0 at the bottom and top interfaces), rho_zz_old_split
    random and rho_zz the density the same fluxes leave after dt (mass-consistent, so the
    upwind update of a constant is that constant), scalars_old random in [0, 0.02] or the
    constant `const`.  Returns (state, cell volumes [nCells, L])."""
    from mpasdyn import mesh as M
    m0 = M.zero_based(mesh)
    st = make_state(m0, L, "physical", seed=seed)
    rng = np.random.default_rng(seed)
    nC, nE = st.nCells, st.nEdges
    lat = st["latEdge"][:nE, 0]
    ang = st["angleEdge"][:nE, 0]
    kk = np.arange(L)[None, :]
    ru = 20.0 * np.cos(lat)[:, None] * np.cos(ang)[:, None] * (1 + 0.5 * np.sin(0.3 * kk)) \
        + 2.0 * rng.standard_normal((nE, L))
    st["ruAvg"][:nE, :L] = ru
    st["ruAvg"][:nE, L] = 0.0
    ww = 0.01 * rng.standard_normal((nC, L + 1))  # vertical Courant number <~ 0.1
    ww[:, 0] = 0.0
    ww[:, L] = 0.0
    st["wwAvg"][:nC] = ww
    ro = 0.8 + 0.4 * rng.random((nC, L))
    st["rho_zz_old_split"][:nC, :L] = ro
    invA = st["invAreaCell"][:nC, 0]
    dv = st["dvEdge"][:nE, 0]
    rdzw = st["rdzw"][:L]
    eoc = st["edgesOnCell"][:nC]
    coe = st["cellsOnEdge"][:nE]
    ne = st["nEdgesOnCell"][:nC, 0]
    div = np.zeros((nC, L))
    for j in range(eoc.shape[1]):
        on = j < ne
        e = np.where(on, eoc[:, j], 0)
        sg = np.where(coe[e, 0] == np.arange(nC), 1.0, -1.0)
        div += np.where(on[:, None], sg[:, None] * dv[e][:, None] * ru[e], 0.0)
    div = div * invA[:, None] + (ww[:, 1:] - ww[:, :L]) * rdzw[None, :]
    st["rho_zz"][:nC, :L] = ro - dt * div
    if const is None:
        st["scalars_old"][:nC, :L] = 0.02 * rng.random((nC, L, 8))
    else:
        st["scalars_old"][:nC, :L] = const
    vol = 1.0 / (invA[:, None] * rdzw[None, :])
    return st, vol


def compare_elementwise(got, ref, rtol, afloor, fields=None, skip=SCRATCH, zero_slot_excluded=()):
    """Per-element comparison: every finite reference element must hold
    |got - ref| <= rtol * |ref| + afloor * max|ref of that field|, NaN / inf at the same places,
    integer fields equal.  Unlike compare_states' normwise rule, an error in a small entry is
    not hidden behind the field's largest one.  Returns (mismatches, worst) where worst maps
    each float field to its largest |got - ref| / (|ref| + afloor max|ref|)."""
    bad, worst = [], {}
    for f in FIELDS:
        if f.name in skip or (fields is not None and f.name not in fields):
            continue
        a, b = got.arrays[f.name], ref.arrays[f.name]
        if f.name in zero_slot_excluded:
            n = got.n_of(f)
            a, b = a[:n], b[:n]
        if f.dtype != np.float64:
            if not np.array_equal(a, b):
                bad.append((f.name, "int mismatch", None))
            continue
        na, nb = np.isnan(a), np.isnan(b)
        if not np.array_equal(na, nb) or not np.array_equal(np.isinf(a), np.isinf(b)):
            bad.append((f.name, "non-finite mask differs", None))
            continue
        fin = np.isfinite(b)
        if not fin.any():
            continue
        aa, bb = a[fin], b[fin]
        scale = float(np.max(np.abs(bb)))
        lim = rtol * np.abs(bb) + afloor * scale
        d = np.abs(aa - bb)
        with np.errstate(divide="ignore", invalid="ignore"):
            r = np.where(lim > 0, d / np.maximum(np.abs(bb) + afloor * scale, 1e-300), np.where(d > 0, np.inf, 0.0))
        worst[f.name] = float(r.max()) if r.size else 0.0
        over = d > lim
        if over.any():
            i = int(np.argmax(np.where(over, d - lim, -np.inf)))
            bad.append((f.name, float(aa[i]), float(bb[i]), int(over.sum())))
    return bad, worst
