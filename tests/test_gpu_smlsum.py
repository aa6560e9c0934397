"""Option "smlsum" (atm_srk3 fast path, reference semantics, with fusesml): set_smlstep's
slope-flux sum over a cell's edges is formed once per step (k_sml_flux -> X_smlS) and each
stage's fused set_smlstep reads that one column instead of u_tend at the cell's edges and
zb_cell / zb3_cell.  The sum replaces a chain of subtractions from w (reassociated): the step
agrees with the literal form to rounding, per element; the decomposed step stays bit-identical
to one context; the keep tails stay exact."""
import threading

import pytest

import oracle as O
from helpers import ZERO_SLOT_WRITTEN, compare_elementwise, compare_states, make_state
from mpasdyn import decomp, lib
from mpasdyn import tasks as T

pytestmark = pytest.mark.gpu


def _run(st, smlsum, schedule=1, n=2, keep_check=0, graph=1):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", 0)
        assert ctx.get_option("smlsum") == 1  # (default on)
        ctx.set_option("smlsum", smlsum)
        ctx.set_option("graph", graph)
        ctx.set_option("keep_check", keep_check)
        ctx.upload(st)
        for _ in range(n):
            T.atm_srk3(ctx, 720.0, schedule)
        ctx.sync()
        ctx.download(got)
    return got


@pytest.mark.parametrize("variant", ["physical", "random"])
@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("schedule", [0, 1])
def test_smlsum_bit_identical(x1_2562, variant, L, schedule):
    """the fast path sums the terms in k_sml_flux's order wherever set_smlstep runs (fused from
    X_smlS, fused inline, the separate task): the same bits with the option on or off"""
    st = make_state(x1_2562, L, variant)
    a = _run(st, 0, schedule)
    b = _run(st, 1, schedule)
    bad = compare_states(b, a, rtol=0.0)
    assert not bad, bad[:6]


def test_fast_set_smlstep_task(x1_2562):
    """the separate task (fast path: summed) against the oracle's literal chain, per element"""
    st = make_state(x1_2562, 56, "physical")
    ref = st.copy()
    O.Oracle(ref).atm_set_smlstep_pert_variables_work()
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", 0)
        ctx.upload(st)
        T.atm_set_smlstep_pert_variables_work(ctx)
        ctx.sync()
        ctx.download(got)
    bad, _ = compare_elementwise(got, ref, rtol=1e-11, afloor=1e-13)
    assert not bad, bad[:6]


def test_smlsum_against_oracle(x1_2562):
    st = make_state(x1_2562, 56, "physical")
    ref = st.copy()
    O.Oracle(ref).atm_srk3(720.0, 1)
    got = _run(st, 1, n=1)
    bad, _ = compare_elementwise(got, ref, rtol=1e-9, afloor=1e-11, zero_slot_excluded=ZERO_SLOT_WRITTEN)
    assert not bad, bad[:6]


def test_smlsum_keep_tails(x1_2562):
    """option keep_check with the fused set_smlstep from X_smlS (eager launches): w's level-L
    tail follows the values it writes"""
    st = make_state(x1_2562, 56, "random")
    a = _run(st, 1, graph=0, keep_check=1)
    b = _run(st, 1)
    assert not compare_states(a, b, rtol=0.0)


@pytest.mark.parametrize("nparts", [2, 3])
def test_smlsum_decomposed_equals_single(x1_2562, nparts):
    """loopback subdomains (X_smlS of the owned cells from u_tend at their ring-1 edges):
    bit-identical to one context with the same option"""
    st = make_state(x1_2562, 56, "random")
    one = _run(st, 1, n=1)
    d = decomp.Decomposition(st, nparts)
    locs = [d.local_state(r) for r in range(nparts)]
    ctxs = [lib.Context(*d.n_local(r), st.L) for r in range(nparts)]
    try:
        for r, c in enumerate(ctxs):
            c.set_option("exact", 0)
            lib.setup_subdomain(c, d, r)
            c.upload(locs[r])
        lib.halo_loopback(ctxs)
        errs = [None] * nparts

        def drive(r):
            try:
                T.atm_srk3(ctxs[r], 720.0, 1)
                ctxs[r].sync()
            except Exception as e:  # noqa: BLE001 -- reported below
                errs[r] = e
        th = [threading.Thread(target=drive, args=(r,)) for r in range(nparts)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert all(e is None for e in errs), errs
        for r, c in enumerate(ctxs):
            c.download(locs[r])
    finally:
        for c in ctxs:
            c.close()
    got = d.assemble(locs)
    bad = compare_states(got, one, rtol=0.0)
    assert not bad, bad[:6]
