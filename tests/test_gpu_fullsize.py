"""Size-independent properties at the benchmark's full size, x1.163842 x 56 levels (the
oracle takes seconds per step there; these checks need no oracle):

* the benchmark path (exact = 0: Q10 as L * sum, acoustic recurrence as a scan) stays
  within the documented 1e-9 of the literal order (exact = 1) over a whole RK3 step;
* a 2- and an 8-subdomain decomposition (loopback transport, halo overlap on) are
  bit-identical to the undecomposed run over a whole RK3 step.

The state is the benchmark's: the mesh and its one-time precompute from the host, the
3-D fields filled on the device by the seeded generator (global ids, so every subdomain
holds the same values as the single run)."""
import os
import sys
import threading

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from mpasdyn import decomp, lib  # noqa: E402
from mpasdyn import tasks as T  # noqa: E402
from mpasdyn.registry import FIELDS  # noqa: E402
from mpasdyn.state import HostState  # noqa: E402

from helpers import compare_states  # noqa: E402

NC, L = 163842, 56
CHECK = ["u", "w", "theta_m", "rho_pp", "rtheta_pp", "rw_p", "ru_p", "tend_u", "tend_theta", "tend_rho",
         "pv_edge", "divergence", "ke", "vorticity", "wwAvg", "ruAvg"]
_KIND = {f.name: f.entity for f in FIELDS}


@pytest.fixture(scope="module")
def workload():
    import bench
    m, st = bench.build_inputs(NC, L)
    return bench, m, st, bench.dt_for(NC)


def run_single(workload, exact):
    bench, m, st, dt = workload
    out = HostState(m.nCells, m.nEdges, m.nVertices, L, names=CHECK)
    with lib.Context(m.nCells, m.nEdges, m.nVertices, L) as ctx:
        ctx.set_option("exact", exact)
        bench.upload_inputs(ctx, st)
        T.atm_srk3(ctx, dt, 1)
        ctx.sync()
        ctx.download(out)
    return out


@pytest.mark.gpu
def test_fullsize_fast_within_tolerance_of_exact(workload):
    fast, exact = run_single(workload, 0), run_single(workload, 1)
    for name in CHECK:
        assert np.isfinite(exact[name]).all(), name
    bad = compare_states(fast, exact, rtol=1e-9, fields=CHECK)
    assert not bad, bad


_REF = {}


@pytest.mark.gpu
@pytest.mark.parametrize("nparts", [2, 8])
def test_fullsize_decomposed_equals_single(workload, nparts):
    """nparts = 8: the decomposition of the 8-GPU benchmark run, its halos moved by the
    loopback transport on one GPU (RCCL itself needs the 8 devices)"""
    bench, m, st, dt = workload
    if "ref" not in _REF:
        _REF["ref"] = run_single(workload, 1)
    ref = _REF["ref"]
    n = nparts
    d = decomp.Decomposition(st, n)
    locs = [d.local_state(r) for r in range(n)]
    ctxs = [lib.Context(*d.n_local(r), L) for r in range(n)]
    outs = [HostState(*d.n_local(r), L, names=CHECK) for r in range(n)]
    try:
        for r, c in enumerate(ctxs):
            c.set_option("exact", 1)
            lib.setup_subdomain(c, d, r)
            bench.upload_inputs(c, locs[r])
        lib.halo_loopback(ctxs)
        errs = [None] * n

        def drive(r):
            try:
                T.atm_srk3(ctxs[r], dt, 1)
                ctxs[r].sync()
            except Exception as e:  # noqa: BLE001 -- reported below
                errs[r] = e
        th = [threading.Thread(target=drive, args=(r,)) for r in range(n)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert errs == [None] * n, errs
        for r, c in enumerate(ctxs):
            c.download(outs[r])
    finally:
        for c in ctxs:
            c.close()
    got = HostState(m.nCells, m.nEdges, m.nVertices, L, names=CHECK)
    for name in CHECK:
        for r in range(n):
            own = d.owned[r][_KIND[name]]
            got.arrays[name][own] = outs[r].arrays[name][:len(own)]
        got.arrays[name][-1] = ref.arrays[name][-1]  # the zero slot is not downloaded by rank
    bad = compare_states(got, ref, rtol=0.0, fields=CHECK)
    assert not bad, bad
