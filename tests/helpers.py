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


def compare_states(got, ref, rtol=0.0, fields=None, skip=SCRATCH, tol_fields=None):
    """Return a list of (field, max_abs_err, scale) mismatches.

    rtol == 0 demands bit-identical arrays (NaNs must sit at the same places).
    Otherwise |got - ref| <= rtol * max|ref| per field (normwise), for the fields in
    tol_fields (all fields when tol_fields is None); the others stay bit-exact."""
    bad = []
    for f in FIELDS:
        if f.name in skip or (fields is not None and f.name not in fields):
            continue
        a, b = got.arrays[f.name], ref.arrays[f.name]
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
