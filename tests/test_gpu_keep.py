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


def _run(st, fn, exact=1, physics=0, transport=0, **opts):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        for k, v in opts.items():
            ctx.set_option(k, v)
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


@pytest.mark.parametrize("opts", [{"hfuse": 0}, {"hfuse": 0, "bsplit": 1}, {"hfuse": 0, "etile": 1},
                                  {"hfuse": 0, "etile": 0}, {"hfuse": 1, "smlsum": 0}],
                         ids=["hfuse0", "hfuse0-bsplit", "hfuse0-etile", "hfuse0-noetile", "hfuse1-nosmlsum"])
def test_keep_srk3_fast(x1_2562, opts):
    """the fast path (exact 0) with the check on, in the large grids' launch order (hfuse 0: the
    separate k_sml_flux and setup launches, B / Bf under bsplit, the tiled E): no kept slot changes
    without its tail, and the step stays within the fast path's tolerance of the oracle"""
    st = make_state(x1_2562, 56, "physical")
    ref = st.copy()
    O.Oracle(ref).atm_srk3(720.0, 1)
    got = _run(st, lambda c: T.atm_srk3(c, 720.0, 1), exact=0, **opts)
    bad = compare_states(got, ref, rtol=1e-9, zero_slot_excluded=ZERO_SLOT_WRITTEN)
    assert not bad, bad[:6]


@pytest.mark.parametrize("physics,transport", [(1, 0), (2, 0), (2, 1)])
def test_keep_srk3_mpas_fast(x1_2562, physics, transport):
    """the MPAS forms' fast path with the check on (bsplit and fusecopy on under physics 2, the
    first ru update k_acoustic_ru<FIRST>, the MPAS set_smlstep), from the balanced JW state (the
    synthetic states blow up under the MPAS forms, beyond any normwise tolerance of the fast path)"""
    from mpasdyn import jw
    st = jw.jw_state(M.zero_based(x1_2562), 26, perturb=True)
    step = lambda c: T.atm_srk3(c, 720.0, 1)  # noqa: E731
    got = _run(st, step, exact=0, physics=physics, transport=transport)
    # the check changes nothing: the same bits as the unchecked, graph-replayed step
    plain = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", 0)
        ctx.set_option("physics", physics)
        ctx.set_option("transport", transport)
        ctx.upload(st)
        step(ctx)
        ctx.sync()
        ctx.download(plain)
    bad = compare_states(got, plain, rtol=0.0)
    assert not bad, bad[:6]
    if physics == 2:  # (physics 1 keeps the reference's dyn_tend: the JW state blows up there)
        ref = st.copy()
        O.Oracle(ref).mpas_srk3(720.0, 1, transport=bool(transport), physics=physics)
        bad = compare_states(got, ref, rtol=1e-9, zero_slot_excluded=ZERO_SLOT_WRITTEN)
        assert not bad, bad[:6]


@pytest.mark.parametrize("exact", [1, 0])
def test_keep_decomposed(x1_2562, exact):
    """loopback subdomains with the check on: the ghosts' kept slots arrive with the exchanged
    columns (the owners' values), the tails of the owned entities stay exact"""
    import threading
    st = make_state(x1_2562, 56, "random")
    if exact:
        ref = st.copy()
        O.Oracle(ref).atm_srk3(720.0, 1)
    else:  # (the fast path: N subdomains give one context's bits; fused damping with its halo)
        ref = _run(st, lambda c: T.atm_srk3(c, 720.0, 1), exact=0)
    d = decomp.Decomposition(st, 3)
    locs = [d.local_state(r) for r in range(3)]
    ctxs = [lib.Context(*d.n_local(r), st.L) for r in range(3)]
    try:
        for r, c in enumerate(ctxs):
            c.set_option("exact", exact)
            c.set_option("keep_check", 1)
            assert c.get_option("fusedamp_halo") == 1
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
