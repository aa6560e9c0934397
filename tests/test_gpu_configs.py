"""Every BASELINE.json configuration on the GPU, against the oracle where the oracle runs
in seconds, and through size-independent properties where it does not.

config 2  x1.2562 x 56                 tests/test_gpu_parity.py (per task and per step)
config 3  x1.40962 x 56, full RK3     one atm_srk3 step vs the oracle (below)
headline  x1.163842 x 56 (config 4's   one atm_srk3 step vs the oracle (below); the
          mesh; 8 GPUs split it)        8-subdomain split: tests/test_gpu_fullsize.py
config 5  x1.655362 x 56 + moist       MPAS-dynamics step with the transport from the JW
          transport, 8 GPUs            state: 8-subdomain loopback split = single context,
                                        bit for bit; the transport task at full size
                                        conserves sum(rho s volume), no new extrema

The bench workload is used as is: the mesh with its one-time precompute from the host,
the 3-D state filled on the device by the seeded generator (bench.upload_inputs).  For
the oracle the device state is downloaded whole right after upload, so both sides start
from the same bits.  Tolerances: exact = 1 bit-identical; the benchmark
path exact = 0 (Q10 as L * sum, the acoustic recurrence as a scan) within 1e-9 of each
field's max magnitude over a whole step.
"""
import os
import sys
import threading

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import oracle as O  # noqa: E402
from mpasdyn import decomp, lib  # noqa: E402
from mpasdyn import tasks as T  # noqa: E402
from mpasdyn.registry import FIELDS  # noqa: E402
from mpasdyn.state import HostState  # noqa: E402

from helpers import compare_states  # noqa: E402

pytestmark = pytest.mark.gpu
L = 56
RTOL_FAST = 1e-9
_KIND = {f.name: f.entity for f in FIELDS}


def _workload(ncells, zero_based=False):
    import bench
    m, st = bench.build_inputs(ncells, L, zero_based=zero_based)
    return bench, m, st, bench.dt_for(ncells)


def _gpu_step(bench, m, st, dt, exact, opts=None, names=None, start=None):
    """upload the bench state, optionally download it whole (`start`), run one step,
    download `names` (None: every field)"""
    out = HostState(m.nCells, m.nEdges, m.nVertices, L, names=names)
    with lib.Context(m.nCells, m.nEdges, m.nVertices, L) as ctx:
        ctx.set_option("exact", exact)
        for k, v in (opts or {}).items():
            ctx.set_option(k, v)
        bench.upload_inputs(ctx, st)
        if start is not None:
            ctx.download(start)
        T.atm_srk3(ctx, dt, 1)
        ctx.sync()
        ctx.download(out)
    return out


@pytest.mark.parametrize("ncells", [40962, 163842])
def test_srk3_step_vs_oracle(ncells):
    """config 3 (x1.40962) and the headline mesh (x1.163842): one RK3 step of the bench
    workload, GPU exact = oracle bit for bit, GPU fast within 1e-9"""
    bench, m, st, dt = _workload(ncells)
    start = HostState(m.nCells, m.nEdges, m.nVertices, L)
    got = _gpu_step(bench, m, st, dt, 1, start=start)
    moved = {n: start[n].copy() for n in ("tend_u", "tend_theta", "rw_p", "rho_pp", "ru_p")}
    ref = start
    O.Oracle(ref).atm_srk3(dt, 1)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]
    del got
    fast = _gpu_step(bench, m, st, dt, 0)
    bad = compare_states(fast, ref, rtol=RTOL_FAST)
    assert not bad, bad[:6]
    # the step did something: the tendencies and the acoustic variables moved
    for name, before in moved.items():
        assert np.any(ref[name] != before), name


CHECK5 = ["u", "w", "theta_m", "rho_zz", "rho_p", "rtheta_p", "exner", "pressure_p", "ru", "rw", "ruAvg", "wwAvg",
          "tend_u", "tend_w", "tend_theta", "pv_edge", "divergence", "ke", "vorticity", "scalars", "surface_pressure"]


def test_config5_transport_step_decomposed_equals_single():
    """config 5 on one GPU: x1.655362 x 56, the MPAS dynamics (physics = 2, which includes
    the vertical solver of physics = 1) with the monotonic transport of 8 scalars inside
    atm_srk3, from the perturbed JW state (a balanced atmosphere: every value finite), split
    into the 8 subdomains of the 8-GPU run with the halo moved by the loopback transport
    (overlap on): bit-identical to the undecomposed context, exact and benchmark paths"""
    from mpasdyn import jw
    from mpasdyn import mesh as M
    m = M.zero_based(M.icosahedral(8))
    st = jw.jw_state(m, L, perturb=True, subset=True, extra_names=("scalars",))
    nC = m.nCells
    st["scalars"][:nC, :L] = 0.02 * np.random.default_rng(5).random((nC, L, 8))
    dt = 720.0 * 2.0 ** (4 - 8)  # 45 s
    opts = {"physics": 2, "transport": 1}
    n = 8
    d = decomp.Decomposition(st, n)
    locs = [d.local_state(r) for r in range(n)]

    def step(c):
        T.atm_compute_solve_diagnostics(c, False, -1)  # MPAS-A's initial diagnostics
        T.mpas_reconstruct_2d(c, False, True)
        T.atm_srk3(c, dt, 1)
        T.atm_compute_output_diagnostics(c)
    for exact in (1, 0):
        ref = HostState(m.nCells, m.nEdges, m.nVertices, L, names=CHECK5)
        with lib.Context(m.nCells, m.nEdges, m.nVertices, L) as ctx:
            ctx.set_option("exact", exact)
            for k, v in opts.items():
                ctx.set_option(k, v)
            ctx.upload(st)
            step(ctx)
            ctx.sync()
            ctx.download(ref)
        for name in CHECK5:
            assert np.isfinite(ref[name][:-1]).all(), name
        sp = ref["surface_pressure"][:nC, 0]
        assert np.abs(sp - 1.0e5).max() < 500.0  # one 45-s step of the (perturbed) JW state
        ctxs = [lib.Context(*d.n_local(r), L) for r in range(n)]
        outs = [HostState(*d.n_local(r), L, names=CHECK5) for r in range(n)]
        try:
            for r, c in enumerate(ctxs):
                c.set_option("exact", exact)
                for k, v in opts.items():
                    c.set_option(k, v)
                lib.setup_subdomain(c, d, r)
                c.upload(locs[r])
            lib.halo_loopback(ctxs)
            errs = [None] * n

            def drive(r):
                try:
                    step(ctxs[r])
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
        got = HostState(m.nCells, m.nEdges, m.nVertices, L, names=CHECK5)
        for name in CHECK5:
            for r in range(n):
                own = d.owned[r][_KIND[name]]
                got.arrays[name][own] = outs[r].arrays[name][:len(own)]
            got.arrays[name][-1] = ref.arrays[name][-1]  # the zero slot is not downloaded by rank
        bad = compare_states(got, ref, rtol=0.0, fields=CHECK5)
        assert not bad, f"exact={exact}: {bad[:6]}"
        del ref, got, outs


TRANSPORT_IN = ["ruAvg", "wwAvg", "rho_zz_old_split", "rho_zz", "scalars_old", "scalars"]


def test_config5_transport_conserves_and_bounds_at_full_size():
    """the transport task at x1.655362 x 56 x 8 scalars (helpers.transport_state's flow,
    built here from the mesh arrays only): sum(rho s volume) conserved to 1e-12 relative
    per scalar, every new value inside the old values of its neighbourhood"""
    import bench
    from mpasdyn import build_state as bs
    from mpasdyn import mesh as M
    m = M.zero_based(M.icosahedral(8))
    st = bs.build_state(m, L, "physical", mesh_only=True)
    nC, nE = st.nCells, st.nEdges
    vals = HostState(nC, nE, st.nVertices, L, names=TRANSPORT_IN)
    rng = np.random.default_rng(20211015)
    lat, ang = st["latEdge"][:nE, 0], st["angleEdge"][:nE, 0]
    kk = np.arange(L)[None, :]
    ru = 20.0 * np.cos(lat)[:, None] * np.cos(ang)[:, None] * (1 + 0.5 * np.sin(0.3 * kk))
    ru += 2.0 * rng.standard_normal((nE, L))
    vals["ruAvg"][:nE, :L] = ru
    ww = 0.01 * rng.standard_normal((nC, L + 1))
    ww[:, 0] = ww[:, L] = 0.0
    vals["wwAvg"][:nC] = ww
    ro = 0.8 + 0.4 * rng.random((nC, L))
    vals["rho_zz_old_split"][:nC, :L] = ro
    invA, dv, rdzw = st["invAreaCell"][:nC, 0], st["dvEdge"][:nE, 0], st["rdzw"][:L]
    eoc, coe, ne = st["edgesOnCell"][:nC], st["cellsOnEdge"][:nE], st["nEdgesOnCell"][:nC, 0]
    div = np.zeros((nC, L))
    for j in range(eoc.shape[1]):
        on = j < ne
        e = np.where(on, eoc[:, j], 0)
        sg = np.where(coe[e, 0] == np.arange(nC), 1.0, -1.0)
        div += np.where(on[:, None], sg[:, None] * dv[e][:, None] * ru[e], 0.0)
    del ru
    dt = bench.dt_for(655362)
    vals["rho_zz"][:nC, :L] = ro - dt * (div * invA[:, None] + (ww[:, 1:] - ww[:, :L]) * rdzw[None, :])
    del div
    s_old = 0.02 * rng.random((nC, L, 8))
    vals["scalars_old"][:nC, :L] = s_old
    with lib.Context(nC, nE, st.nVertices, L) as ctx:
        ctx.set_option("physics", 1)
        bench.upload_inputs(ctx, st)
        ctx.upload(vals, names=TRANSPORT_IN)
        T.atm_advance_scalars_mono(ctx, dt)
        ctx.sync()
        ctx.download(vals, names=["scalars"])
    s_new = vals["scalars"][:nC, :L]
    vol = 1.0 / (invA[:, None] * rdzw[None, :])
    m_old = np.einsum("ck,cki->i", ro * vol, s_old)
    m_new = np.einsum("ck,cki->i", vals["rho_zz"][:nC, :L] * vol, s_new)
    assert np.allclose(m_new, m_old, rtol=1e-12, atol=0), (m_new, m_old)
    lo, hi = s_old.copy(), s_old.copy()
    lo[:, 1:] = np.minimum(lo[:, 1:], s_old[:, :-1])
    hi[:, 1:] = np.maximum(hi[:, 1:], s_old[:, :-1])
    lo[:, :-1] = np.minimum(lo[:, :-1], s_old[:, 1:])
    hi[:, :-1] = np.maximum(hi[:, :-1], s_old[:, 1:])
    for j in range(eoc.shape[1]):
        on = j < ne
        e = np.where(on, eoc[:, j], 0)
        c1, c2 = coe[e, 0], coe[e, 1]
        oth = np.where(on, np.where(c1 == np.arange(nC), c2, c1), np.arange(nC))
        np.minimum(lo, s_old[oth], out=lo)
        np.maximum(hi, s_old[oth], out=hi)
    eps = 1e-13 * 0.02
    assert np.all(s_new >= lo - eps) and np.all(s_new <= hi + eps)
    assert np.any(s_new != s_old)
