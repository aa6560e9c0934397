"""Keep tails (round 5, mpas_dev.h): the slots the reference never writes -- level L of most
task outputs, level 0 of vert_imp's tridiagonal coefficients -- are now written with the value
they hold, read from a per-field tail, so that every 128-B line of a column is written whole.
Option "keep_check" compares every tail with its field after every task; these runs fail the
task on any mismatch (a kernel that changed a kept slot without its tail), and the results
stay bit-identical to the oracle (exact mode).  The state variants put random values in the
kept slots, so a stale tail would also show as a value difference."""
import pytest

import oracle as O
from helpers import ZERO_SLOT_WRITTEN, compare_states, make_state
from mpasdyn import decomp, lib
from mpasdyn import mesh as M
from mpasdyn import tasks as T
from test_gpu_parity import TASKS

pytestmark = pytest.mark.gpu


def _run(st, fn, exact=1, physics=0, transport=0):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", exact)
        ctx.set_option("graph", 0)  # (the check runs between eager launches)
        ctx.set_option("physics", physics)
        ctx.set_option("transport", transport)
        ctx.set_option("keep_check", 1)
        assert ctx.get_option("keep_check") == 1
        ctx.upload(st)
        fn(ctx)
        ctx.sync()
        ctx.download(got)
    return got


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("task", TASKS, ids=[t[0] for t in TASKS])
def test_keep_tasks(x1_2562, L, task):
    name, ofn, gfn, _ = task
    st = make_state(x1_2562, L, "random")
    ref = st.copy()
    ofn(O.Oracle(ref))
    got = _run(st, gfn)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, f"{name}: {bad[:6]}"


@pytest.mark.parametrize("variant", ["random", "mpas0"])
@pytest.mark.parametrize("schedule", [0, 1])
def test_keep_srk3(x1_2562, variant, schedule):
    m = M.zero_based(x1_2562) if variant == "mpas0" else x1_2562
    st = make_state(m, 56, "random")
    ref = st.copy()
    o = O.Oracle(ref)
    for _ in range(2):
        o.atm_srk3(720.0, schedule)
    got = _run(st, lambda c: [T.atm_srk3(c, 720.0, schedule) for _ in range(2)])
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("physics,transport", [(1, 0), (2, 0), (1, 1), (2, 1)])
def test_keep_srk3_mpas(x1_2562, physics, transport):
    st = make_state(M.zero_based(x1_2562), 26, "random")
    ref = st.copy()
    O.Oracle(ref).mpas_srk3(720.0, 1, transport=bool(transport), physics=physics)
    got = _run(st, lambda c: T.atm_srk3(c, 720.0, 1), physics=physics, transport=transport)
    bad = compare_states(got, ref, rtol=1e-14, tol_fields={"exner", "pressure_p"}, zero_slot_excluded=ZERO_SLOT_WRITTEN)
    assert not bad, bad[:6]


def test_keep_decomposed(x1_2562):
    """loopback subdomains with the check on: the ghosts' kept slots arrive with the exchanged
    columns (the owners' values), the tails of the owned entities stay exact"""
    import threading
    st = make_state(x1_2562, 56, "random")
    ref = st.copy()
    O.Oracle(ref).atm_srk3(720.0, 1)
    d = decomp.Decomposition(st, 3)
    locs = [d.local_state(r) for r in range(3)]
    ctxs = [lib.Context(*d.n_local(r), st.L) for r in range(3)]
    try:
        for r, c in enumerate(ctxs):
            c.set_option("exact", 1)
            c.set_option("keep_check", 1)
            lib.setup_subdomain(c, d, r)
            c.upload(locs[r])
        lib.halo_loopback(ctxs)
        errs = [None] * 3

        def drive(r):
            try:
                T.atm_srk3(ctxs[r], 720.0, 1)
                ctxs[r].sync()
            except Exception as e:  # noqa: BLE001 -- reported below
                errs[r] = e
        th = [threading.Thread(target=drive, args=(r,)) for r in range(3)]
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
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]
