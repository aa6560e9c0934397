"""Option "etile": dyn_tend's cell kernel E over compact tiles of cells, each tile's theta_m
closure staged in LDS and every edge's advCells flux formed there (k_dyn_Et) -- the edge kernel B
then forms no flux and the per-edge scratch X_F goes.  The flux is B's expression in B's order
and the per-cell sums are E's, so the tiled path gives the same bits as the untiled one in both
the exact and the fast mode, and the exact mode stays bit-identical to the oracle
(dynamics_tasks.rg:1328-1360)."""
import numpy as np
import pytest

import oracle as O
from helpers import ZERO_SLOT_WRITTEN, compare_states, make_state
from mpasdyn import mesh as M
from mpasdyn import tasks as T
from mpasdyn import lib

pytestmark = pytest.mark.gpu


def _run(st, etile, exact, fn, **opts):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", exact)
        ctx.set_option("etile", etile)
        for k, v in opts.items():
            ctx.set_option(k, v)
        ctx.upload(st)
        fn(ctx)
        ctx.sync()
        active = ctx.get_option("etile_active")
        ctx.download(got)
    return got, active


@pytest.mark.parametrize("variant", ["random", "physical"])
@pytest.mark.parametrize("exact", [0, 1])
@pytest.mark.parametrize("L", [40, 56])
def test_etile_steps_bit_identical(x1_2562, L, exact, variant):
    st = make_state(x1_2562, L, variant)
    steps = lambda ctx: [T.atm_srk3(ctx, 720.0, 1) for _ in range(2)]  # noqa: E731
    a, act0 = _run(st, 0, exact, steps)
    b, act1 = _run(st, 1, exact, steps)
    assert act0 == 0 and act1 == 1  # (LP = 64, reference semantics, undecomposed: tiles built)
    bad = compare_states(b, a, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("rk_step", [0, 1])
@pytest.mark.parametrize("exact", [0, 1])
def test_etile_dyn_tend_task(x1_2562, rk_step, exact):
    """the task alone (B with D at rk_step 0, E's rk_step > 0 perturbation flux): tiled = untiled,
    and in exact mode = the oracle bit for bit"""
    st = make_state(x1_2562, 56, "random")
    task = lambda ctx: T.atm_compute_dyn_tend_work(ctx, rk_step, 720.0)  # noqa: E731
    a, _ = _run(st, 0, exact, task)
    b, act = _run(st, 1, exact, task)
    assert act == 1
    bad = compare_states(b, a, rtol=0.0)
    assert not bad, bad[:6]
    if exact:
        ref = st.copy()
        O.Oracle(ref).atm_compute_dyn_tend_work(rk_step, 720.0)
        bad = compare_states(b, ref, rtol=0.0)
        assert not bad, bad[:6]


@pytest.mark.parametrize("cells,clo", [(1, 20), (4, 40), (8, 56), (16, 96), (40, 160)])
def test_etile_tile_sizes(x1_2562, cells, clo):
    """any tile size limit gives the same bits (one cell per tile up to the largest closure)"""
    st = make_state(x1_2562, 56, "physical")
    steps = lambda ctx: T.atm_srk3(ctx, 720.0, 1)  # noqa: E731
    a, _ = _run(st, 0, 0, steps)
    b, act = _run(st, 1, 0, steps, etcells=cells, etclo=clo)
    assert act == 1
    bad = compare_states(b, a, rtol=0.0)
    assert not bad, bad[:6]


def test_etile_against_oracle_step(x1_2562):
    """the fast path with tiles stays within the fast path's tolerance of the oracle"""
    st = make_state(x1_2562, 56, "physical")
    ref = st.copy()
    O.Oracle(ref).atm_srk3(720.0, 1)
    got, act = _run(st, 1, 0, lambda ctx: T.atm_srk3(ctx, 720.0, 1))
    assert act == 1
    bad = compare_states(got, ref, rtol=1e-9, zero_slot_excluded=ZERO_SLOT_WRITTEN)
    assert not bad, bad[:6]
    assert np.isfinite(got["u"]).all()


def test_etile_inactive_where_unsupported(x1_2562):
    """no tiles below LP = 64 or under the MPAS dynamics (the untiled kernels run)"""
    for L, physics, mesh in ((5, 0, x1_2562), (56, 2, M.zero_based(x1_2562))):
        st = make_state(mesh, L, "physical")
        with lib.Context(*st.dims()) as ctx:
            ctx.set_option("physics", physics)
            ctx.set_option("etile", 1)
            ctx.upload(st)
            assert ctx.get_option("etile_active") == 0


def test_etile_keep_check_fast(x1_2562):
    """keep tails under the tiled fast path (exact 0, eager steps: every task checked)"""
    st = make_state(x1_2562, 56, "random")
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", 0)
        ctx.set_option("etile", 1)
        ctx.set_option("graph", 0)
        ctx.set_option("keep_check", 1)
        ctx.upload(st)
        T.atm_srk3(ctx, 720.0, 1)
        ctx.sync()


# ---------------------------------------------------------------- option ntu
# (2: stage 1's solve_diagnostics stores every diagnostic; 3: the stages' last substeps store the acoustic state)
@pytest.mark.parametrize("ntu", [1, 2, 3])
@pytest.mark.parametrize("hfuse", [0, 2])  # (0: the large grids' launches, stage 0's solve_diagnostics skipped)
@pytest.mark.parametrize("variant", ["random", "physical"])
@pytest.mark.parametrize("exact", [0, 1])
@pytest.mark.parametrize("L", [5, 56])
def test_ntu_steps_bit_identical(x1_2562, L, exact, variant, hfuse, ntu):
    """option ntu (atm_srk3, defer4 out): rk_step 0's edge kernel forms no tend_u -- dead there, the
    next stage's edge kernel rewrites it and no task in between reads it -- so every field after the
    step, tend_u included, has the same bits with the option on and off; exact mode = the oracle"""
    st = make_state(x1_2562, L, variant)
    steps = lambda ctx: [T.atm_srk3(ctx, 720.0, 1) for _ in range(2)]  # noqa: E731
    a, _ = _run(st, 0, exact, steps, ntu=0, hfuse=hfuse)
    b, _ = _run(st, 0, exact, steps, ntu=ntu, hfuse=hfuse)
    bad = compare_states(b, a, rtol=0.0)
    assert not bad, bad[:6]
    if exact:
        ref = st.copy()
        o = O.Oracle(ref)
        for _ in range(2):
            o.atm_srk3(720.0, 1)
        bad = compare_states(b, ref, rtol=0.0)
        assert not bad, bad[:6]


def test_ntu_only_where_dead(x1_2562):
    """the standalone task (no next stage) and the reference's driver schedule (schedule 0: no
    rk_step 0 stage) keep the whole tend_u: the same bits as the oracle with the option on"""
    st = make_state(x1_2562, 56, "random")
    got, _ = _run(st, 0, 1, lambda ctx: T.atm_compute_dyn_tend_work(ctx, 0, 720.0), ntu=1)
    ref = st.copy()
    O.Oracle(ref).atm_compute_dyn_tend_work(0, 720.0)
    assert not compare_states(got, ref, rtol=0.0)
    # (dt = 1: stages 0 and 1 at rk_step 0, Q4 -- stage 0's solve is live; dt = 0.5: every stage at
    # rk_step 0 -- stage 1's whole solve is live too)
    for dt in (720.0, 1.0, 0.5):
        got, _ = _run(st, 0, 1, lambda ctx: T.atm_srk3(ctx, dt, 0), ntu=1, hfuse=0)
        ref = st.copy()
        O.Oracle(ref).atm_srk3(dt, 0)
        assert not compare_states(got, ref, rtol=0.0)
