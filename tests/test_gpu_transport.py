"""GPU (libmpasdyn k_transport.hip) vs oracle parity of the monotonic scalar transport
(Q26: no reference transport exists, the oracle restates MPAS-A's
atm_advance_scalars_mono and is pinned by tests/test_transport.py's properties).

Tolerances: the kernels evaluate the oracle's expressions in its operand order (built
with -ffp-contract=off), so the task is value-identical to the oracle.  Inside a whole
RK3 step with physics = 1 the inputs come from the dynamics: exact mode is
value-identical except the pow fields (RTOL_POW), fast mode within RTOL_STEP = 1e-9.
"""
import numpy as np
import pytest

import oracle as O
from helpers import ZERO_SLOT_WRITTEN, compare_states, make_state, transport_state
from mpasdyn import lib, tasks as T

pytestmark = pytest.mark.gpu

DT = 600.0
RTOL_STEP = 1e-9
RTOL_POW = 1e-14
POW_FIELDS = {"exner", "pressure_p"}


def gpu(st, fn, exact=1, physics=1, transport=0, trorder=None, trsu=0, trepw=1):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", exact)
        ctx.set_option("physics", physics)
        ctx.set_option("transport", transport)
        if trorder is not None:  # (None: the library default, 64)
            ctx.set_option("trorder", trorder)
        ctx.set_option("trsu", trsu)
        ctx.set_option("trepw", trepw)
        ctx.upload(st)
        fn(ctx)
        ctx.sync()
        ctx.download(got)
    return got


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("const", [None, 0.0123])
def test_transport_task(x1_2562, L, const):
    st, vol = transport_state(x1_2562, L, DT, const=const)
    ref = st.copy()
    O.Oracle(ref).mpas_advance_scalars_mono(DT)
    got = gpu(st, lambda c: T.atm_advance_scalars_mono(c, DT))
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]
    # and the properties hold on the GPU result
    nC = st.nCells
    m_old = np.einsum("ck,cki->i", st["rho_zz_old_split"][:nC, :L] * vol, st["scalars_old"][:nC, :L])
    m_new = np.einsum("ck,cki->i", got["rho_zz"][:nC, :L] * vol, got["scalars"][:nC, :L])
    assert np.allclose(m_new, m_old, rtol=1e-12, atol=0)


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("trorder,trsu,trepw", [(0, 0, 1), (1, 0, 1), (7, 0, 1), (256, 0, 1), (0, 1, 1), (64, 1, 1),
                                                (0, 0, 2), (7, 0, 2), (64, 0, 2), (-256, 0, 1), (-1, 0, 2)])
def test_transport_task_pair_major(x1_2562, L, trorder, trsu, trepw):
    """option trorder = 0 (entity-major), 1 (pair-major slot order) and R >= 2 (pair-major
    within runs of R entities, the last run partial at R = 7 and 256); option trsu (su formed again by the
    update instead of stored): speed only, the same values"""
    st, _ = transport_state(x1_2562, L, DT)
    ref = st.copy()
    O.Oracle(ref).mpas_advance_scalars_mono(DT)
    if trorder < 0:  # option trorder_e (the edge kernel's own order) beside the default trorder
        def run(c):
            c.set_option("trorder_e", -trorder)
            T.atm_advance_scalars_mono(c, DT)
        got = gpu(st, run, trsu=trsu, trepw=trepw)
    else:
        got = gpu(st, lambda c: T.atm_advance_scalars_mono(c, DT), trorder=trorder, trsu=trsu, trepw=trepw)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("L", [1, 2, 63])
def test_transport_task_edge_levels(x1_2562, L):
    """nVertLevels 1 (no interior interface), 2 (2nd-order only), 63 (LP 64, full column)"""
    st, _ = transport_state(x1_2562, L, DT)
    ref = st.copy()
    O.Oracle(ref).mpas_advance_scalars_mono(DT)
    got = gpu(st, lambda c: T.atm_advance_scalars_mono(c, DT))
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


def test_transport_task_random_ids(x1_2562):
    """the literal 1-based ids of the reference's mesh (cells not among their edges'
    cells: the non-SELF gathers) and every input synthetic"""
    st = make_state(x1_2562, 5, "random")
    ref = st.copy()
    O.Oracle(ref).mpas_advance_scalars_mono(DT)
    got = gpu(st, lambda c: T.atm_advance_scalars_mono(c, DT))
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("L", [5, 56])
def test_srk3_transport(x1_2562, L):
    """option transport = 1: scalars saved to scalars_old, then the transport after the
    last stage's recover, inside mpas_atm_srk3"""
    from mpasdyn import mesh as M
    st = make_state(M.zero_based(x1_2562), L, "random")
    ref = st.copy()
    O.Oracle(ref).mpas_srk3(720.0, 1, transport=True)
    assert not np.array_equal(ref["scalars"], st["scalars"])
    for exact, tol, tf in ((1, RTOL_POW, POW_FIELDS), (0, RTOL_STEP, None)):
        got = gpu(st, lambda c: T.atm_srk3(c, 720.0, 1), exact=exact, transport=1)
        bad = compare_states(got, ref, rtol=tol, tol_fields=tf, zero_slot_excluded=ZERO_SLOT_WRITTEN)
        assert not bad, f"exact={exact}: {bad[:6]}"


def test_transport_option_rules(x1_2562):
    st = make_state(x1_2562, 5, "random")
    with lib.Context(*st.dims()) as ctx:
        with pytest.raises(lib.MpasError):
            ctx.set_option("transport", 1)  # needs physics = 1
        ctx.set_option("physics", 1)
        ctx.set_option("transport", 1)
        assert ctx.get_option("transport") == 1
        ctx.set_option("physics", 0)
        assert ctx.get_option("transport") == 0


def _with(opts, fn):
    def g(c):
        for k, v in opts.items():
            c.set_option(k, v)
        fn(c)
    return g


@pytest.mark.parametrize("nparts", [2, 3])
@pytest.mark.parametrize("overlap", [1, 0])
@pytest.mark.parametrize("trtile,trsu,trepw", [(0, 0, 1), (1, 0, 1), (0, 1, 1), (0, 0, 2)])
def test_transport_decomposed_equals_single(x1_2562, nparts, overlap, trtile, trsu, trepw):
    """N subdomains (loopback halo: the x8 fields move as 8 columns per entity) give the
    single-context result bit for bit, with the three kernels and with the tiles (whose
    interior launch takes only the cells reading owned columns)"""
    from test_gpu_decomp import run_decomposed, run_single
    st, _ = transport_state(x1_2562, 56, DT)
    def step(c):
        if c.get_option("trtile_ghosts"):  # a decomposed context: the tiles must be in use
            assert c.get_option("trtile_active") == trtile
        T.atm_advance_scalars_mono(c, DT)
    fn = _with({"physics": 1, "trtile": trtile, "trsu": trsu, "trepw": trepw}, step)
    ref = run_single(st, fn, 1)
    got, stats = run_decomposed(st, nparts, fn, 1, overlap=overlap, tiled_transport=bool(trtile))
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]
    assert all(s[0] > 0 for s in stats)


@pytest.mark.parametrize("L", [5, 56])
def test_srk3_transport_decomposed(x1_2562, L):
    from mpasdyn import mesh as M
    from test_gpu_decomp import run_decomposed, run_single
    st = make_state(M.zero_based(x1_2562), L, "random")
    fn = _with({"physics": 1, "transport": 1}, lambda c: T.atm_srk3(c, 720.0, 1))
    for exact in (1, 0):
        ref = run_single(st, fn, exact)
        got, _ = run_decomposed(st, 3, fn, exact)
        bad = compare_states(got, ref, rtol=0.0)
        assert not bad, f"exact={exact}: {bad[:6]}"


@pytest.mark.parametrize("L", [5, 56])
def test_tiled_equals_three_kernel(x1_2562, L):
    """option trtile = 1 (opt-in: the two tiled kernels, k_trt_*) against trtile = 0 (the
    three kernels with the edge scratch): bit for bit; the tiles are active on the x1 mesh"""
    st, _ = transport_state(x1_2562, L, DT)
    outs = {}
    for tile in (0, 1):
        got = st.copy()
        with lib.Context(*st.dims()) as ctx:
            ctx.set_option("physics", 1)
            ctx.set_option("trtile", tile)
            ctx.upload(st)
            assert ctx.get_option("trtile_active") == tile
            if tile:
                assert 0 < ctx.get_option("trtile_count") <= st.nCells
            T.atm_advance_scalars_mono(ctx, DT)
            ctx.sync()
            ctx.download(got)
        outs[tile] = got
    bad = compare_states(outs[1], outs[0], rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("variant", ["mesh", "random"])
@pytest.mark.parametrize("L", [56, 63])
def test_edge_groups_equal_direct(x1_2562, variant, L):
    """option tredge (opt-in, LP 64): k_tr_edge_lds, the edge kernel with each group's
    scalars_old columns staged in LDS, against tredge = 0 (k_tr_edge's direct gathers) and
    the oracle: bit for bit; random ids make irregular groups (too large a union: direct
    gathers inside the same kernel)"""
    if variant == "mesh":
        st, _ = transport_state(x1_2562, L, DT)
    else:
        st = make_state(x1_2562, L, "random")
    ref = st.copy()
    O.Oracle(ref).mpas_advance_scalars_mono(DT)
    outs = {}
    for on in (0, 1):
        got = st.copy()
        with lib.Context(*st.dims()) as ctx:
            ctx.set_option("physics", 1)
            ctx.set_option("tredge", on)
            ctx.upload(st)
            assert ctx.get_option("tredge_active") == on
            if on and variant == "random":
                assert ctx.get_option("tredge_irregular") > 0
            T.atm_advance_scalars_mono(ctx, DT)
            ctx.sync()
            ctx.download(got)
        outs[on] = got
    bad = compare_states(outs[1], outs[0], rtol=0.0)
    assert not bad, bad[:6]
    bad = compare_states(outs[1], ref, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("physics", [1, 2])
@pytest.mark.parametrize("L", [5, 56])
def test_trsave_bit_identical(x1_2562, physics, L):
    """option trsave (atm_srk3 with the transport): scalars_save's copy folded into the transport --
    its edge and bounds kernels read the old scalars from scalars, the bounds kernel stores every
    level of each pair column (and the zero slot's) to scalars_old -- the same bits in every field,
    scalars_old included, as the separate copy; two steps, exact and fast"""
    from mpasdyn import mesh as M
    st = make_state(M.zero_based(x1_2562), L, "random")
    for exact in (1, 0):
        out = {}
        for save in (0, 1):
            got = st.copy()
            with lib.Context(*st.dims()) as ctx:
                ctx.set_option("exact", exact)
                ctx.set_option("physics", physics)
                ctx.set_option("transport", 1)
                ctx.set_option("trsave", save)
                ctx.upload(st)
                for _ in range(2):
                    T.atm_srk3(ctx, 720.0, 1)
                ctx.sync()
                ctx.download(got)
            out[save] = got
        bad = compare_states(out[1], out[0], rtol=0.0)
        assert not bad, f"exact={exact}: {bad[:6]}"
        assert np.array_equal(out[1]["scalars_old"], out[0]["scalars_old"])
