"""The MPAS dynamics (option physics = 2) on the GPU against the oracle (ora_mpas_*,
pinned on the CPU by tests/test_mpas_dynamics.py: JW balance, mass, wave growth).

Per task on synthetic states (x1.2562, raw 1-based ids "random" and 0-based "mpas0", 5 and
56 levels): exact mode value-identical; the acoustic step's fast path (two affine scans)
and dyn_tend's (theta and w fluxes summed per edge) within RTOL_FAST.  Whole RK3 steps: exact
mode value-identical except the two fields that
go through pow in recover (RTOL_POW), fast mode within RTOL_STEP.

JW day 1 (the north star's check, BASELINE.json: surface pressure within 1e-10 relative):
120 steps of 720 s from the JW state on x1.2562 x 26 on the GPU against the same 120
oracle steps: day-1 surface pressure within 1e-10 relative (exact and benchmark paths);
the reference itself never changes surface pressure (Q7), so this compares with the
MPAS dynamics restated in the oracle (parity unpinned against the Regent run)."""
import numpy as np
import pytest

import oracle as O
from helpers import ZERO_SLOT_WRITTEN, compare_states, make_state
from mpasdyn import jw, lib
from mpasdyn import mesh as M
from mpasdyn import tasks as T

pytestmark = pytest.mark.gpu

RTOL_FAST = 1e-11
RTOL_STEP = 1e-9
RTOL_POW = 1e-14
RTOL_EXTREME = 1e-6
POW_FIELDS = {"exner", "pressure_p"}
ACOUSTIC_FIELDS = {"rho_pp", "rtheta_pp", "rw_p", "wwAvg"}
# the fast path forms the theta and w fluxes per edge in dyn_tend's edge kernel and sums them
# per cell (reassociated): these fields agree to RTOL_FAST, the rest stay value-identical
DYN_FIELDS = {"tend_theta", "tend_rtheta_adv", "rthdynten", "tend_w"}

_ST = {}


def state(mesh, L, variant):
    key = (L, variant)
    if key not in _ST:
        m = M.zero_based(mesh) if variant == "mpas0" else mesh
        st = make_state(m, L, "random")
        O.Oracle(st).mpas_vert_imp_coefs(240.0)  # a factored system for the acoustic step
        _ST[key] = st
    return _ST[key]


def run_gpu(st, fn, exact, transport=0):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", exact)
        ctx.set_option("physics", 2)
        ctx.set_option("transport", transport)
        ctx.upload(st)
        fn(ctx)
        ctx.sync()
        ctx.download(got)
    return got


def run_oracle(st, fn):
    ref = st.copy()
    fn(O.Oracle(ref))
    return ref


def _out_diag(o):
    o.atm_compute_output_diagnostics()
    o.mpas_surface_pressure()


TASKS = [
    ("setup", lambda o: o.mpas_rk_integration_setup(), lambda c: T.atm_rk_integration_setup(c), set()),
    ("moist", lambda o: o.mpas_moist_coefficients(), lambda c: T.atm_compute_moist_coefficients(c), set()),
    ("dyn_tend_rk0", lambda o: o.mpas_dyn_tend(0, 720.0), lambda c: T.atm_compute_dyn_tend_work(c, 0, 720.0), DYN_FIELDS),
    ("dyn_tend_rk1", lambda o: o.mpas_dyn_tend(1, 720.0), lambda c: T.atm_compute_dyn_tend_work(c, 1, 720.0), DYN_FIELDS),
    ("dyn_tend_rk2_rayleigh", lambda o: o.mpas_dyn_tend(2, 720.0, config_rayleigh_damp_u=True),
     lambda c: T.atm_compute_dyn_tend_work(c, 2, 720.0, config_rayleigh_damp_u=True), DYN_FIELDS),
    ("dyn_tend_rk0_fixed_cam", lambda o: o.mpas_dyn_tend(0, 720.0, "2d_fixed", 0.5),
     lambda c: T.atm_compute_dyn_tend_work(c, 0, 720.0, "2d_fixed", 0.5), DYN_FIELDS),
    ("smlstep", lambda o: o.mpas_set_smlstep(), lambda c: T.atm_set_smlstep_pert_variables_work(c), set()),
    ("acoustic_s0", lambda o: o.mpas2_acoustic_step(240.0, 0), lambda c: T.atm_advance_acoustic_step_work(c, 240.0, 0),
     ACOUSTIC_FIELDS),
    ("acoustic_s1", lambda o: o.mpas2_acoustic_step(360.0, 1), lambda c: T.atm_advance_acoustic_step_work(c, 360.0, 1),
     ACOUSTIC_FIELDS),
    ("solve_diag_rk0", lambda o: o.mpas_solve_diagnostics(0, 0), lambda c: T.atm_compute_solve_diagnostics(c, False, 0),
     set()),
    ("solve_diag_rk2", lambda o: o.mpas_solve_diagnostics(0, 2), lambda c: T.atm_compute_solve_diagnostics(c, False, 2),
     set()),
    ("finish", lambda o: o.mpas_substep_finish(1, 1), lambda c: T.atm_rk_dynamics_substep_finish(c, 1, 1), set()),
    ("output_diagnostics", _out_diag, lambda c: T.atm_compute_output_diagnostics(c), set()),
]


@pytest.mark.parametrize("L", [1, 2, 5, 56, 63])
@pytest.mark.parametrize("variant", ["random", "mpas0"])
@pytest.mark.parametrize("task", TASKS, ids=[t[0] for t in TASKS])
def test_task(x1_2562, L, variant, task):
    name, ofn, gfn, tol_fields = task
    st = state(x1_2562, L, variant)
    ref = run_oracle(st, ofn)
    got = run_gpu(st, gfn, 1)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, f"{name} exact: {bad[:6]}"
    got.check_zero_slots()
    if tol_fields:
        got = run_gpu(st, gfn, 0)
        bad = compare_states(got, ref, rtol=RTOL_FAST, tol_fields=tol_fields)
        assert not bad, f"{name} fast: {bad[:6]}"


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("transport", [0, 1])
def test_srk3(x1_2562, L, transport):
    st = state(x1_2562, L, "mpas0")
    ref = run_oracle(st, lambda o: o.mpas_srk3(720.0, 1, transport=bool(transport), physics=2))
    for exact, tol, tf in ((1, RTOL_POW, POW_FIELDS), (0, RTOL_STEP, None)):
        got = run_gpu(st, lambda c: T.atm_srk3(c, 720.0, 1), exact, transport)
        bad = compare_states(got, ref, rtol=tol, tol_fields=tf, zero_slot_excluded=ZERO_SLOT_WRITTEN)
        assert not bad, f"exact={exact}: {bad[:6]}"


def _jw(x1_2562, L, perturb=False):
    st = jw.jw_state(M.zero_based(x1_2562), L, perturb=perturb)
    o = O.Oracle(st)
    o.mpas_solve_diagnostics(0, -1)
    o.mpas_reconstruct_2d(False, True)
    return st


@pytest.mark.parametrize("perturb", [False, True])
def test_jw_day1_surface_pressure(x1_2562, perturb):
    """one simulated day (120 x 720 s) from the JW state: the GPU's day-1 surface pressure
    equals the oracle's within 1e-10 relative, in the exact and in the benchmark path"""
    L, n = 26, 120
    st = _jw(x1_2562, L, perturb)
    ref = st.copy()
    o = O.Oracle(ref)
    for _ in range(n):
        o.mpas_srk3(720.0, 1, physics=2)
    o.atm_compute_output_diagnostics()
    o.mpas_surface_pressure()
    nC = st.nCells
    sp_ref = ref["surface_pressure"][:nC, 0].copy()
    assert np.isfinite(sp_ref).all() and np.abs(sp_ref - 1.0e5).max() < 100.0 + 400.0 * perturb
    for exact in (1, 0):
        got = st.copy()
        with lib.Context(*st.dims()) as ctx:
            ctx.set_option("exact", exact)
            ctx.set_option("physics", 2)
            ctx.upload(st)
            for _ in range(n):
                T.atm_srk3(ctx, 720.0, 1)
            T.atm_compute_output_diagnostics(ctx)
            ctx.sync()
            ctx.download(got)
        sp = got["surface_pressure"][:nC, 0]
        rel = np.abs(sp - sp_ref).max() / np.abs(sp_ref).max()
        assert rel <= 1e-10, f"exact={exact}: day-1 surface pressure differs by {rel:.3e} relative"
        bad = compare_states(got, ref, rtol=1e-8, fields=["u", "w", "theta_m", "rho_zz", "pressure_p"], zero_slot_excluded=ZERO_SLOT_WRITTEN)
        assert not bad, f"exact={exact}: {bad[:6]}"


def test_driver_day1(x1_2562):
    """python -m mpasdyn.driver --physics 2 --day: the end-to-end run reports the day-1
    surface pressure (balanced within 1 hPa) and a conserved dry mass"""
    from mpasdyn import driver
    lines = []
    st = driver.run(x1_2562, 26, 120, 720.0, physics=2, out=None, log=lines.append)
    sp = st["surface_pressure"][:st.nCells, 0]
    assert np.isfinite(sp).all() and np.abs(sp - 1.0e5).max() < 100.0
    assert "surface pressure" in lines[-1] and "dry mass change" in lines[-1]
    assert abs(float(lines[-1].split("dry mass change ")[1])) < 1e-12


@pytest.mark.parametrize("nparts", [2, 3])
def test_decomposed_equals_single(x1_2562, nparts):
    """physics = 2 on N subdomains (loopback halo, overlap on): bit-identical to the single
    context over an RK3 step of the JW state (every new gather of the mode is declared)"""
    from test_gpu_decomp import run_decomposed, run_single

    def fn(c):
        c.set_option("physics", 2)
        T.atm_compute_solve_diagnostics(c, False, -1)
        T.mpas_reconstruct_2d(c, False, True)
        T.atm_srk3(c, 720.0, 1)
        T.atm_srk3(c, 720.0, 1)
    st = jw.jw_state(M.zero_based(x1_2562), 26, perturb=True)
    for exact in (1, 0):
        ref = run_single(st, fn, exact)
        got, stats = run_decomposed(st, nparts, fn, exact)
        bad = compare_states(got, ref, rtol=0.0)
        assert not bad, f"exact={exact}: {bad[:6]}"


@pytest.mark.parametrize("L", [1, 2, 63])
@pytest.mark.parametrize("physics", [1, 2])
def test_srk3_level_extremes(x1_2562, L, physics):
    """the MPAS forms (physics 1: the vertical solver, 2: also the dynamics) with the
    transport at nVertLevels 1, 2 (degenerate vertical stencils and tridiagonal systems)
    and 63 (LP = 64, level L in the last lane): a whole RK3 step against the oracle, exact
    (pow fields RTOL_POW) and fast (RTOL_EXTREME: the synthetic state is no atmosphere --
    at 63 levels its fields reach 1e18 within the step and the scan's rounding differences
    grow with them, to 5e-7 of a field's magnitude in h_divergence)"""
    st = state(x1_2562, L, "mpas0")
    ref = run_oracle(st, lambda o: o.mpas_srk3(720.0, 1, transport=True, physics=physics))
    for exact, tol, tf in ((1, RTOL_POW, POW_FIELDS), (0, RTOL_EXTREME, None)):
        got = st.copy()
        with lib.Context(*st.dims()) as ctx:
            ctx.set_option("exact", exact)
            ctx.set_option("physics", physics)
            ctx.set_option("transport", 1)
            ctx.upload(st)
            T.atm_srk3(ctx, 720.0, 1)
            ctx.sync()
            ctx.download(got)
        bad = compare_states(got, ref, rtol=tol, tol_fields=tf, zero_slot_excluded=ZERO_SLOT_WRITTEN)
        assert not bad, f"L={L} physics={physics} exact={exact}: {bad[:6]}"


@pytest.mark.parametrize("physics", [1, 2])
@pytest.mark.parametrize("L", [5, 56])
def test_mpas_fusesetup_bit_identical(x1_2562, physics, L):
    """atm_srk3 under the MPAS solver / dynamics with option fusesetup (setup + moist + vert_imp
    of stage 0 in one launch, with the MPAS forms: vert_imp's LU, theta_m_save and cqu by the
    edge blocks) equals the separate launches bit for bit, in the exact and the fast path, with
    the transport under physics 1"""
    st = state(x1_2562, L, "mpas0")
    for exact in (1, 0):
        out = {}
        for fused in (1, 0):
            got = st.copy()
            with lib.Context(*st.dims()) as ctx:
                ctx.set_option("exact", exact)
                ctx.set_option("physics", physics)
                ctx.set_option("transport", 1 if physics == 1 else 0)
                ctx.set_option("fusesetup", fused)
                ctx.upload(st)
                for _ in range(3):
                    T.atm_srk3(ctx, 720.0, 1)
                ctx.sync()
                ctx.download(got)
            out[fused] = got
        bad = compare_states(out[1], out[0], rtol=0.0)
        assert not bad, f"exact={exact}: {bad[:6]}"


@pytest.mark.parametrize("physics,transport", [(1, 1), (2, 0), (2, 1)])
@pytest.mark.parametrize("L", [5, 56])
def test_ntu_mpas_forms_bit_identical(x1_2562, physics, transport, L):
    """option ntu under the MPAS forms: the stages before the last recover no ruAvg / wwAvg (the next
    stage's first acoustic substep sets both before any task reads them) and their solve_diagnostics
    store ke, pv_edge and rho_edge alone (divergence, vorticity, h_edge and ke_edge have no reader
    before the last stage's call rewrites them) -- every field after three steps, the transport's
    scalars included, has the same bits with the option on and off (2, 3: each part alone)"""
    st = state(x1_2562, L, "mpas0")
    for exact in (1, 0):
        out = {}
        for ntu in (0, 1, 2, 3):
            got = st.copy()
            with lib.Context(*st.dims()) as ctx:
                ctx.set_option("exact", exact)
                ctx.set_option("physics", physics)
                ctx.set_option("transport", transport)
                ctx.set_option("ntu", ntu)
                ctx.upload(st)
                for _ in range(3):
                    T.atm_srk3(ctx, 720.0, 1)
                ctx.sync()
                ctx.download(got)
            out[ntu] = got
        for ntu in (1, 2, 3):
            bad = compare_states(out[ntu], out[0], rtol=0.0)
            assert not bad, f"exact={exact} ntu={ntu}: {bad[:6]}"


@pytest.mark.parametrize("physics,transport", [(1, 1), (2, 0)])
@pytest.mark.parametrize("L", [5, 56])
def test_mdamp_bit_identical(x1_2562, physics, transport, L):
    """option mdamp (the MPAS forms): each divergence damping applied by the kernel that next reads
    ru_p -- the next substep's ru_p kernel, or the stage's recover edge kernel (before its cell kernel
    rewrites theta_m; rho_zz of the edge's cells formed as that kernel forms it) -- instead of a launch
    of its own: every field after three steps (number_of_sub_steps 2: a damping inside a stage and at
    each stage's end) has the same bits as the separate launches, with ntu on and off"""
    st = state(x1_2562, L, "mpas0")
    for exact in (1, 0):
        out = {}
        for mdamp, ntu in ((0, 0), (1, 0), (1, 1)):
            got = st.copy()
            with lib.Context(*st.dims()) as ctx:
                ctx.set_option("exact", exact)
                ctx.set_option("physics", physics)
                ctx.set_option("transport", transport)
                ctx.set_option("mdamp", mdamp)
                ctx.set_option("ntu", ntu)
                ctx.upload(st)
                for _ in range(3):
                    T.atm_srk3(ctx, 720.0, 1)
                ctx.sync()
                ctx.download(got)
            out[(mdamp, ntu)] = got
        for key in ((1, 0), (1, 1)):
            bad = compare_states(out[key], out[(0, 0)], rtol=0.0)
            assert not bad, f"exact={exact} mdamp, ntu={key}: {bad[:6]}"


@pytest.mark.parametrize("transport", [0, 1])
@pytest.mark.parametrize("L", [5, 56])
def test_mru_bit_identical(x1_2562, transport, L):
    """option mru (the MPAS dynamics, fast path): the kernel forming each stage's final tend_u (B, or D
    at rk_step 0) also stores the first acoustic substep's ru_p = dts tend_u and ruAvg = ru_p, and that
    substep's ru_p kernel goes -- every field after three steps has the same bits as with the kernel"""
    st = state(x1_2562, L, "mpas0")
    out = {}
    for mru in (0, 1):
        got = st.copy()
        with lib.Context(*st.dims()) as ctx:
            ctx.set_option("exact", 0)
            ctx.set_option("physics", 2)
            ctx.set_option("transport", transport)
            ctx.set_option("mru", mru)
            ctx.upload(st)
            for _ in range(3):
                T.atm_srk3(ctx, 720.0, 1)
            ctx.sync()
            ctx.download(got)
        out[mru] = got
    bad = compare_states(out[1], out[0], rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("transport", [0, 1])
@pytest.mark.parametrize("L", [5, 56])
def test_msml_bit_identical(x1_2562, transport, L):
    """option msml (the MPAS dynamics): each stage's set_smlstep applied by dyn_tend's E to the tend_w
    it forms (k_set_smlstep's loads and order of operations) instead of a launch of its own -- every
    field after three steps has the same bits, exact and fast"""
    st = state(x1_2562, L, "mpas0")
    for exact in (1, 0):
        out = {}
        for msml in (0, 1):
            got = st.copy()
            with lib.Context(*st.dims()) as ctx:
                ctx.set_option("exact", exact)
                ctx.set_option("physics", 2)
                ctx.set_option("transport", transport)
                ctx.set_option("msml", msml)
                ctx.upload(st)
                for _ in range(3):
                    T.atm_srk3(ctx, 720.0, 1)
                ctx.sync()
                ctx.download(got)
            out[msml] = got
        bad = compare_states(out[1], out[0], rtol=0.0)
        assert not bad, f"exact={exact}: {bad[:6]}"
