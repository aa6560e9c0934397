"""GPU (libmpasdyn, gfx950) vs oracle parity, per task and for the whole RK3 step.

Inputs: x1.2562 (the reference's own mesh, raw ids, Q1 zero slots) at the repo-default
5 levels and at 56 levels, in two state variants -- "random" (every input synthetic,
flags and masks random: every branch and term runs on non-zero data) and "ref" (the
literal reference state: Q2 fields zero, init restatements).

Tolerances (stated here, per SURVEY §8.4 and BASELINE.json's 1e-10 relative):
* exact mode (mpas_set_option("exact", 1)): every field value-identical to the oracle.
  The library is built with -ffp-contract=off and evaluates each expression in the
  Regent operand order, so nothing is reassociated.
* fast mode (the benchmark path): the reassociated computations differ by rounding
  only -- q (Q10, nVertLevels*term instead of nVertLevels additions), the theta flux of
  dyn_tend summed per edge in B (H = ru F + dvEdge (ru_save - ru) theta_m_save, E sums
  edgesOnCell_sign H) and the acoustic recurrence (affine prefix scan over the column).  Their outputs must agree to
  RTOL_FAST = 1e-11 relative to the field's max magnitude; all other fields of a single
  task stay value-identical.  Across a whole RK3 step the differences propagate, and
  every field is held to RTOL_STEP = 1e-9.
"""
import numpy as np
import pytest

import oracle as O
from helpers import ZERO_SLOT_WRITTEN, SCRATCH, compare_states, make_state
from mpasdyn import lib, tasks as T

pytestmark = pytest.mark.gpu

RTOL_FAST = 1e-11
RTOL_STEP = 1e-9
# downstream of q, and of the theta flux H that the fast path forms per edge in B
Q_FIELDS = {"tend_u", "tend_u_euler", "tend_theta", "tend_rtheta_adv", "rthdynten"}
ACOUSTIC_FIELDS = {"rho_pp", "rtheta_pp", "rw_p", "wwAvg"}

# (id, oracle call, gpu call, fields the fast path may round differently)
TASKS = [
    ("setup", lambda o: o.atm_rk_integration_setup(), lambda c: T.atm_rk_integration_setup(c), set()),
    ("moist", lambda o: o.atm_compute_moist_coefficients(), lambda c: T.atm_compute_moist_coefficients(c), set()),
    ("vert_imp", lambda o: o.atm_compute_vert_imp_coefs(240.0), lambda c: T.atm_compute_vert_imp_coefs(c, 240.0), set()),
    ("dyn_tend_rk0", lambda o: o.atm_compute_dyn_tend_work(0, 720.0),
     lambda c: T.atm_compute_dyn_tend_work(c, 0, 720.0), Q_FIELDS),
    ("dyn_tend_rk1", lambda o: o.atm_compute_dyn_tend_work(1, 720.0),
     lambda c: T.atm_compute_dyn_tend_work(c, 1, 720.0), Q_FIELDS),
    ("dyn_tend_rk2_rayleigh", lambda o: o.atm_compute_dyn_tend_work(2, 720.0, config_rayleigh_damp_u=True),
     lambda c: T.atm_compute_dyn_tend_work(c, 2, 720.0, config_rayleigh_damp_u=True), Q_FIELDS),
    ("dyn_tend_rk0_fixed_cam", lambda o: o.atm_compute_dyn_tend_work(0, 720.0, "2d_fixed", 0.5),
     lambda c: T.atm_compute_dyn_tend_work(c, 0, 720.0, "2d_fixed", 0.5), Q_FIELDS),
    ("smlstep", lambda o: o.atm_set_smlstep_pert_variables_work(),
     lambda c: T.atm_set_smlstep_pert_variables_work(c), set()),
    ("acoustic_s0", lambda o: o.atm_advance_acoustic_step_work(240.0, 0),
     lambda c: T.atm_advance_acoustic_step_work(c, 240.0, 0), ACOUSTIC_FIELDS),
    ("acoustic_s1", lambda o: o.atm_advance_acoustic_step_work(360.0, 1),
     lambda c: T.atm_advance_acoustic_step_work(c, 360.0, 1), ACOUSTIC_FIELDS),
    ("div_damp", lambda o: o.atm_divergence_damping_3d(240.0), lambda c: T.atm_divergence_damping_3d(c, 240.0), set()),
    ("solve_diag_rk0", lambda o: o.atm_compute_solve_diagnostics(0, 0),
     lambda c: T.atm_compute_solve_diagnostics(c, False, 0), set()),
    ("solve_diag_rk2", lambda o: o.atm_compute_solve_diagnostics(0, 2),
     lambda c: T.atm_compute_solve_diagnostics(c, False, 2), set()),
    ("solve_diag_holl", lambda o: o.atm_compute_solve_diagnostics(1, -1),
     lambda c: T.atm_compute_solve_diagnostics(c, True, -1), set()),
    ("finish_1_1", lambda o: o.atm_rk_dynamics_substep_finish(1, 1), lambda c: T.atm_rk_dynamics_substep_finish(c, 1, 1),
     set()),
    ("finish_1_2", lambda o: o.atm_rk_dynamics_substep_finish(1, 2), lambda c: T.atm_rk_dynamics_substep_finish(c, 1, 2),
     set()),
    ("finish_2_2", lambda o: o.atm_rk_dynamics_substep_finish(2, 2), lambda c: T.atm_rk_dynamics_substep_finish(c, 2, 2),
     set()),
    ("output_diagnostics", lambda o: o.atm_compute_output_diagnostics(), lambda c: T.atm_compute_output_diagnostics(c),
     set()),
]

_STATES = {}


def base_state(mesh, L, variant):
    """variants: "random", "ref" (build_state) and "mpas0" -- the random state on the
    same mesh with mpas-mode (0-based) ids, where every cell is among the cellsOnEdge of
    its edges and the cell kernels take the SELF gathers (mpas_get_option "selfc")"""
    key = (L, variant)
    if key not in _STATES:
        if variant == "mpas0":
            from mpasdyn import mesh as M
            _STATES[key] = make_state(M.zero_based(mesh), L, "random")
        else:
            _STATES[key] = make_state(mesh, L, variant)
    return _STATES[key]


def run_gpu(st, fn, exact):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", exact)
        ctx.upload(st)
        fn(ctx)
        ctx.sync()
        ctx.download(got)
    return got


def run_oracle(st, fn):
    ref = st.copy()
    fn(O.Oracle(ref))
    return ref


@pytest.mark.parametrize("L", [1, 2, 5, 56, 63])
@pytest.mark.parametrize("variant", ["random", "ref", "mpas0"])
@pytest.mark.parametrize("task", TASKS, ids=[t[0] for t in TASKS])
def test_task_exact(x1_2562, L, variant, task):
    name, ofn, gfn, _ = task
    st = base_state(x1_2562, L, variant)
    ref = run_oracle(st, ofn)
    got = run_gpu(st, gfn, exact=1)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, f"{name}: GPU differs from oracle: {bad[:6]}"
    got.check_zero_slots()


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("task", [t for t in TASKS if t[3]], ids=[t[0] for t in TASKS if t[3]])
@pytest.mark.parametrize("variant", ["random", "mpas0"])
def test_task_fast(x1_2562, L, variant, task):
    name, ofn, gfn, tol_fields = task
    st = base_state(x1_2562, L, variant)
    ref = run_oracle(st, ofn)
    got = run_gpu(st, gfn, exact=0)
    bad = compare_states(got, ref, rtol=RTOL_FAST, tol_fields=tol_fields)
    assert not bad, f"{name}: fast path outside {RTOL_FAST}: {bad[:6]}"


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("variant", ["random", "ref", "mpas0"])
@pytest.mark.parametrize("schedule", [0, 1])
def test_srk3(x1_2562, L, variant, schedule):
    st = base_state(x1_2562, L, variant)
    ref = run_oracle(st, lambda o: o.atm_srk3(720.0, schedule))
    got = run_gpu(st, lambda c: T.atm_srk3(c, 720.0, schedule), exact=1)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, f"srk3 exact: {bad[:6]}"
    got = run_gpu(st, lambda c: T.atm_srk3(c, 720.0, schedule), exact=0)
    bad = compare_states(got, ref, rtol=RTOL_STEP)
    assert not bad, f"srk3 fast: {bad[:6]}"


def test_timestep_dt_zero_nan(x1_2562):
    """Q3: main.rg:66 passes dt = j, so the first step has dt = 0: rdts = inf in the
    divergence damping (:1737) makes ru_p NaN/inf exactly where the oracle has them."""
    st = base_state(x1_2562, 5, "ref")
    ref = run_oracle(st, lambda o: o.atm_srk3(0.0, 0))
    got = run_gpu(st, lambda c: T.atm_timestep(c, 0.0), exact=1)
    assert np.isnan(ref["ru_p"]).any() or np.isinf(ref["ru_p"]).any()
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, f"dt=0 step: {bad[:6]}"


@pytest.mark.parametrize("variant,expect", [("ref", 0), ("random", 0), ("mpas0", 1)])
def test_self_gathers_detected(x1_2562, variant, expect):
    """the SELF gathers switch on exactly for meshes whose cells are among the
    cellsOnEdge of their own edges (raw 1-based ids shift every neighbour: off)"""
    st = base_state(x1_2562, 5, variant)
    with lib.Context(*st.dims()) as ctx:
        ctx.upload(st)
        assert ctx.get_option("selfc") == expect
        ctx.set_option("self", 0)
        assert ctx.get_option("selfc") == 0


def test_self_gathers_identical(x1_2562):
    """SELF on and off give value-identical results over a whole step (mpas0 mesh)"""
    st = base_state(x1_2562, 56, "mpas0")
    outs = []
    for on in (1, 0):
        got = st.copy()
        with lib.Context(*st.dims()) as ctx:
            ctx.set_option("self", on)
            ctx.upload(st)
            T.atm_srk3(ctx, 720.0, 1)
            ctx.sync()
            ctx.download(got)
        outs.append(got)
    bad = compare_states(outs[0], outs[1], rtol=0.0)
    assert not bad, f"SELF on/off differ: {bad[:6]}"



# ---- operators beside the RK3 loop (not run by atm_srk3) ------------------------------
RTOL_POW = 1e-14  # exner/pressure_p go through pow (device libm vs glibc: a few ulp)
POW_FIELDS = {"exner", "pressure_p"}


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("variant", ["random", "ref", "mpas0"])
@pytest.mark.parametrize("ns,rk_step", [(1, 0), (2, 1), (3, 2)])
def test_recover_large_step(x1_2562, L, variant, ns, rk_step):
    """dynamics_tasks.rg:1766-1872, Q24 literal; the garbage-cell rho_zz = 1.0 lands in
    the zero slot exactly as in the oracle"""
    st = base_state(x1_2562, L, variant)
    ref = run_oracle(st, lambda o: o.atm_recover_large_step_variables_work(ns, rk_step, 240.0))
    n = st.nCells
    # downloads cover the n entities, not the zero slot: the device's zero-slot rho_zz is
    # checked through u, which reads it at every edge whose (raw) cellsOnEdge is n
    assert variant == "mpas0" or (st["cellsOnEdge"][:st.nEdges] == n).any()
    for exact in (1, 0):
        got = run_gpu(st, lambda c: T.atm_recover_large_step_variables_work(c, ns, rk_step, 240.0), exact=exact)
        bad = compare_states(got, ref, rtol=RTOL_POW, tol_fields=POW_FIELDS, zero_slot_excluded=ZERO_SLOT_WRITTEN)
        assert not bad, f"recover ns={ns} rk={rk_step}: {bad[:6]}"
        got.check_zero_slots(written=("rho_zz",))
    assert (ref["rho_zz"][st.nCells, :L] == 1.0).all()


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("variant", ["random", "ref", "mpas0"])
@pytest.mark.parametrize("on_a_sphere", [True, False])
def test_reconstruct_2d(x1_2562, L, variant, on_a_sphere):
    """dynamics_tasks.rg:1893-1948: value-identical (cos/sin of lat/lon from the host libm)"""
    st = base_state(x1_2562, L, variant)
    ref = run_oracle(st, lambda o: o.mpas_reconstruct_2d(False, on_a_sphere))
    got = run_gpu(st, lambda c: T.mpas_reconstruct_2d(c, False, on_a_sphere), exact=0)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, f"reconstruct_2d: {bad[:6]}"
    got.check_zero_slots()


def _summary_gpu(st, detailed, global_vel):
    with lib.Context(*st.dims()) as ctx:
        ctx.upload(st)
        out = T.summarize_timestep(ctx, detailed, global_vel)
    return out


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("case", ["random", "ref", "nan", "ties"])
def test_summarize_timestep(x1_2562, L, case):
    """rk_timestep.rg:29-359: the printed values, bit-identical.  "nan" puts NaNs into w
    and u (the regentlib min/max fold restarts after the last NaN; the first-extreme
    search skips them); "ties" makes the extremes occur many times (first point wins in
    the detailed search, the later point in the fold)."""
    st = base_state(x1_2562, L, "ref" if case == "ref" else "random").copy()
    nC, nE = st.nCells, st.nEdges
    if case == "nan":
        rng = np.random.default_rng(1)
        for name, n in (("w", nC), ("u", nE)):
            a = st[name]
            for _ in range(5):
                a[rng.integers(n), rng.integers(L)] = np.nan
    if case == "ties":
        st["w"][:nC, :L] = np.round(st["w"][:nC, :L] * 2.0) / 2.0
        st["u"][:nE, :L] = np.round(st["u"][:nE, :L] / 20.0) * 20.0
        st["w"][7, 0] = -0.0
    for detailed, global_vel in ((1, 1), (1, 0), (0, 1), (0, 0)):
        ref = O.Oracle(st.copy()).summarize_timestep(detailed, global_vel)
        got = _summary_gpu(st, detailed, global_vel)
        assert np.array_equal(np.isnan(got), np.isnan(ref)), (detailed, global_vel)
        ok = np.where(np.isnan(ref), True, (got == ref) & (np.signbit(got) == np.signbit(ref)))
        assert ok.all(), f"summarize {case} {detailed}{global_vel}: {np.nonzero(~ok)[0]} {got[~ok]} vs {ref[~ok]}"


# ---- edge cases: the smallest and the largest column the device layout holds -----------
@pytest.mark.parametrize("L", [1, 2, 63])
@pytest.mark.parametrize("variant", ["random", "ref"])
def test_srk3_level_extremes(x1_2562, L, variant):
    """nVertLevels = 1 and 2 (most vertical stencils degenerate: flux3 never applies, the
    acoustic recurrence is empty) and 63 (LP = 64: level L sits in the last lane of the
    wavefront, every shuffle edge case at the top); whole RK3 steps, exact and fast"""
    st = make_state(x1_2562, L, variant)
    ref = run_oracle(st, lambda o: o.atm_srk3(720.0, 1))
    got = run_gpu(st, lambda c: T.atm_srk3(c, 720.0, 1), exact=1)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, f"L={L} exact: {bad[:6]}"
    got = run_gpu(st, lambda c: T.atm_srk3(c, 720.0, 1), exact=0)
    bad = compare_states(got, ref, rtol=RTOL_STEP)
    assert not bad, f"L={L} fast: {bad[:6]}"


def test_nonfinite_inputs_propagate(x1_2562):
    """NaN and inf in the state propagate through a step exactly where the oracle puts
    them (the select-based accumulations must not swallow or invent non-finite values)"""
    st = make_state(x1_2562, 5, "random").copy()
    st["theta_m"][17, 2] = np.nan
    st["u"][333, 1] = np.inf
    st["rw"][1200, 3] = -np.inf
    st["pressure_p"][2000, 0] = np.nan
    ref = run_oracle(st, lambda o: o.atm_srk3(720.0, 1))
    got = run_gpu(st, lambda c: T.atm_srk3(c, 720.0, 1), exact=1)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]
    assert np.isnan(ref["tend_theta"]).any()


# ---------------------------------------------------------------- the MPAS vertical solver
def run_gpu_mpas(st, fn, exact):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", exact)
        ctx.set_option("physics", 1)
        ctx.upload(st)
        fn(ctx)
        ctx.sync()
        ctx.download(got)
    return got


def mpas_solver_state(mesh, L, variant):
    st = base_state(mesh, L, variant).copy()
    O.Oracle(st).mpas_vert_imp_coefs(240.0)  # a factored system for the acoustic step
    return st


@pytest.mark.parametrize("L", [5, 56, 63])
@pytest.mark.parametrize("variant", ["random", "mpas0"])
def test_mpas_vert_imp(x1_2562, L, variant):
    """option physics = 1: b_tri with cofwt(k-1) and the LU recurrence of the call"""
    st = base_state(x1_2562, L, variant)
    ref = run_oracle(st, lambda o: o.mpas_vert_imp_coefs(240.0))
    for exact in (1, 0):
        got = run_gpu_mpas(st, lambda c: T.atm_compute_vert_imp_coefs(c, 240.0), exact)
        bad = compare_states(got, ref, rtol=0.0)
        assert not bad, f"exact={exact}: {bad[:6]}"


@pytest.mark.parametrize("L", [5, 56, 63])
@pytest.mark.parametrize("variant", ["random", "mpas0"])
@pytest.mark.parametrize("small_step", [0, 1])
def test_mpas_acoustic(x1_2562, L, variant, small_step):
    """option physics = 1: ru_p update, MPAS order, up and down sweeps of the tridiagonal
    solve (exact: level by level, bit-identical; fast: two affine scans, 1e-11)"""
    st = mpas_solver_state(x1_2562, L, variant)
    ref = run_oracle(st, lambda o: o.mpas_acoustic_step(240.0, small_step))
    for exact, tol in ((1, 0.0), (0, RTOL_FAST)):
        got = run_gpu_mpas(st, lambda c: T.atm_advance_acoustic_step_work(c, 240.0, small_step), exact)
        bad = compare_states(got, ref, rtol=tol)
        assert not bad, f"exact={exact}: {bad[:6]}"


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("variant", ["random", "mpas0"])
@pytest.mark.parametrize("ns,rk_step", [(2, 0), (3, 2)])
def test_mpas_recover(x1_2562, L, variant, ns, rk_step):
    """option physics = 1: recover with Q24 fixed (exner/pressure_p through pow: 1e-14)"""
    st = base_state(x1_2562, L, variant)
    ref = run_oracle(st, lambda o: o.mpas_recover(ns, rk_step, 240.0))
    got = run_gpu_mpas(st, lambda c: T.atm_recover_large_step_variables_work(c, ns, rk_step, 240.0), 1)
    bad = compare_states(got, ref, rtol=RTOL_POW, tol_fields=POW_FIELDS, zero_slot_excluded=ZERO_SLOT_WRITTEN)
    assert not bad, bad[:6]


@pytest.mark.parametrize("L", [5, 56])
def test_mpas_srk3(x1_2562, L):
    """option physics = 1: the MPAS vertical solver, Q5 substeps and recover in the loop"""
    st = base_state(x1_2562, L, "mpas0")
    ref = run_oracle(st, lambda o: o.mpas_srk3(720.0, 1))
    for exact, tol, tf in ((1, RTOL_POW, POW_FIELDS), (0, RTOL_STEP, None)):
        got = run_gpu_mpas(st, lambda c: T.atm_srk3(c, 720.0, 1), exact)
        bad = compare_states(got, ref, rtol=tol, tol_fields=tf, zero_slot_excluded=ZERO_SLOT_WRITTEN)
        assert not bad, f"exact={exact}: {bad[:6]}"


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("variant", ["random", "ref", "mpas0"])
@pytest.mark.parametrize("task", ["damping", "init_coupled"])
def test_init_tasks(x1_2562, L, variant, task):
    """the one-time tasks of atm_core_init on the device (dynamics_tasks.rg:274, :651):
    value-identical except the libm results (sin, pow: device vs glibc, RTOL_POW)"""
    ofn, gfn, tf = {
        "damping": (lambda o: o.atm_compute_damping_coefs(22000.0, 0.2),
                    lambda c: T.atm_compute_damping_coefs(c, 22000.0, 0.2), {"dss"}),
        "init_coupled": (lambda o: o.atm_init_coupled_diagnostics(), lambda c: T.atm_init_coupled_diagnostics(c),
                         {"exner", "exner_base", "pressure_p", "pressure_base"}),
    }[task]
    st = base_state(x1_2562, L, variant).copy()
    if task == "damping":  # a monotone column so the damping layer exists (zd = 22 km)
        st["zgrid"][:st.nCells] = np.linspace(0.0, 30000.0, L + 1)[None, :]
    ref = run_oracle(st, ofn)
    got = run_gpu(st, gfn, exact=1)
    bad = compare_states(got, ref, rtol=RTOL_POW, tol_fields=tf)
    assert not bad, bad[:6]
    if task == "damping":
        assert np.any(ref["dss"][:st.nCells] > 0)


MESH_TASKS = {
    "signs": (lambda o: o.atm_compute_signs(), lambda c: T.atm_compute_signs(c), set()),
    "adv_coef": (lambda o: o.atm_adv_coef_compression(), lambda c: T.atm_adv_coef_compression(c), set()),
    "couple": (lambda o: o.atm_couple_coef_3rd_order(0.25), lambda c: T.atm_couple_coef_3rd_order(c, 0.25), set()),
    "mesh_scaling": (lambda o: o.atm_compute_mesh_scaling(True), lambda c: T.atm_compute_mesh_scaling(c, True),
                     {"meshScalingDel2", "meshScalingDel4"}),
}


@pytest.mark.parametrize("variant", ["random", "ref", "mpas0"])
@pytest.mark.parametrize("task", list(MESH_TASKS))
def test_mesh_tasks(x1_2562, variant, task):
    """the mesh tasks of atm_core_init (dynamics_tasks.rg:46, :133, :303, :595) on the
    device: value-identical to the oracle (mesh scaling: pow of the device vs glibc,
    RTOL_POW); deriv_two (never initialised by the reference) random so that every
    coefficient term is exercised, kiteForCell pre-set (kept where no vertex matches)"""
    ofn, gfn, tf = MESH_TASKS[task]
    st = base_state(x1_2562, 5, variant).copy()
    nE = st.nEdges
    st["deriv_two"][:nE] = np.random.default_rng(7).standard_normal((nE, 30))
    st["kiteForCell"][:st.nCells] = 7
    ref = run_oracle(st, ofn)
    got = run_gpu(st, gfn, exact=1)
    bad = compare_states(got, ref, rtol=RTOL_POW, tol_fields=tf or None) if tf else compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("variant", ["random", "ref", "mpas0"])
def test_atm_core_init(x1_2562, variant):
    """mpas_atm_core_init = the device tasks of atm_core_init in the reference's order"""
    st = base_state(x1_2562, 56, variant).copy()
    st["zgrid"][:st.nCells] = np.linspace(0.0, 30000.0, 57)[None, :]
    ref = run_oracle(st, lambda o: o.atm_core_init())
    got = run_gpu(st, lambda c: T.atm_core_init(c), exact=1)
    tf = {"dss", "exner", "exner_base", "pressure_p", "pressure_base", "uReconstructX", "uReconstructY",
          "uReconstructZ", "uReconstructZonal", "uReconstructMeridional", "meshScalingDel2", "meshScalingDel4"}
    bad = compare_states(got, ref, rtol=RTOL_POW, tol_fields=tf)
    assert not bad, bad[:6]


@pytest.mark.parametrize("field,width", [("nEdgesOnCell", 10), ("nEdgesOnEdge", 20), ("nAdvCellsForEdge", 15)])
def test_upload_rejects_overlong_lists(x1_2562, field, width):
    """a list length past its row width (the kernels' tail loops would read past the row)
    is refused at the boundary; the row width itself is accepted"""
    st = base_state(x1_2562, 5, "mpas0").copy()
    with lib.Context(*st.dims()) as ctx:
        st[field][3, 0] = width
        ctx.upload(st, names=[field])
        st[field][3, 0] = width + 1
        with pytest.raises(lib.MpasError, match="exceeds its list width"):
            ctx.upload(st, names=[field])


# ---- option fusedamp: the damping inside the next acoustic launch ------------------------
def _two_steps_gpu(st, fusedamp, exact, graph=1, fusesetup=None, tmedge=None, fusesml=None, hfuse=None,
                   fusecopy=None, defer4=None, vdyn=None):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", exact)
        ctx.set_option("fusedamp", fusedamp)
        ctx.set_option("hfuse", fusedamp if hfuse is None else hfuse)
        ctx.set_option("fusesml", fusedamp if fusesml is None else fusesml)
        ctx.set_option("fusesetup", fusedamp if fusesetup is None else fusesetup)
        ctx.set_option("tmedge", fusedamp if tmedge is None else tmedge)
        ctx.set_option("fusecopy", fusedamp if fusecopy is None else fusecopy)
        ctx.set_option("defer4", fusedamp if defer4 is None else defer4)
        ctx.set_option("vdyn", fusedamp if vdyn is None else vdyn)
        ctx.set_option("graph", graph)
        ctx.upload(st)
        assert ctx.get_option("fusedamp_active") == fusedamp
        T.atm_srk3(ctx, 720.0, 0)
        T.atm_srk3(ctx, 360.0, 1)
        T.atm_srk3(ctx, 360.0, 1)  # (graph replay of the second capture)
        ctx.sync()
        ctx.download(got)
        orph = ctx.get_option("orphan_edges")
    return got, orph


@pytest.mark.parametrize("L", [1, 2, 5, 56, 63])
@pytest.mark.parametrize("variant", ["random", "ref", "mpas0"])
def test_fusedamp_bit_identical(x1_2562, L, variant):
    """atm_srk3 with six of its seven dampings applied inside the next acoustic launch
    (k_acoustic MODE 2: the same expression on the same values), stage 0's setup, moist
    and vert_imp in one launch (k_setup_vi), each stage's set_smlstep inside its first
    acoustic launch (option fusesml), setup's edge copies made by stage 0's dyn_tend edge
    kernel (option fusecopy; stage 0 runs rk_step > 0 kernels under schedule 0, which read
    ru_save), rk_step 0's dyn_tend D applied by stage 1's edge kernel (option defer4), stage 2's v
    stored by its dyn_tend edge kernel (option vdyn), theta_m(cell2) + theta_m(cell1) per edge taken
    from dyn_tend's edge kernel (option tmedge) and independent neighbouring kernels
    sharing a launch (option hfuse; with fusedamp and without tmedge also a stage's last
    acoustic launch beside its solve_diagnostics vertex / cell kernel and its edge kernel
    beside the next stage's dyn_tend A) is value-identical to the separate launches and
    to the oracle, in exact mode and on the fast path; raw 1-based ids leave edge 0 listed
    by no cell (an orphan, written by the launch's extra blocks)"""
    st = base_state(x1_2562, L, variant)
    ref = run_oracle(st, lambda o: (o.atm_srk3(720.0, 0), o.atm_srk3(360.0, 1), o.atm_srk3(360.0, 1)))
    got1, orph = _two_steps_gpu(st, 1, 1)
    bad = compare_states(got1, ref, rtol=0.0)
    assert not bad, f"fusedamp exact vs oracle: {bad[:6]}"
    if variant == "ref":
        assert orph >= 1
    if variant == "mpas0":
        assert orph == 0
    for graph in (1, 0):
        a, _ = _two_steps_gpu(st, 1, 0, graph)
        b, _ = _two_steps_gpu(st, 0, 0, graph)
        bad = compare_states(a, b, rtol=0.0)
        assert not bad, f"fusedamp fast path vs separate damping (graph={graph}): {bad[:6]}"
    c, _ = _two_steps_gpu(st, 0, 0, 1, fusesetup=1)
    bad = compare_states(c, b, rtol=0.0)
    assert not bad, f"fusesetup alone vs separate launches: {bad[:6]}"
    for hf in (0, 1):  # combined launches of independent kernels with and without the damping fusion
        c, _ = _two_steps_gpu(st, hf, 0, 1, hfuse=1 - hf)
        bad = compare_states(c, b, rtol=0.0)
        assert not bad, f"hfuse={1 - hf}, fusedamp={hf} vs separate launches: {bad[:6]}"
    for ex in (0, 1):  # hfuse with fusedamp and without tmedge: the acoustic + solve_vc and
        # solve_e + next stage's dyn_tend A (+ vert_imp) combined launches
        c, _ = _two_steps_gpu(st, 1, ex, 1, tmedge=0, hfuse=1)
        bad = compare_states(c, b if ex == 0 else ref, rtol=0.0)
        assert not bad, f"hfuse=1, tmedge=0, exact={ex}: {bad[:6]}"
    for fc in (0, 1):  # setup's edge copies in the setup launch / in dyn_tend, exact and fast
        for ex in (0, 1):
            c, _ = _two_steps_gpu(st, 1, ex, 1, fusecopy=fc)
            bad = compare_states(c, b if ex == 0 else ref, rtol=0.0)
            assert not bad, f"fusecopy={fc}, exact={ex}: {bad[:6]}"
    for vd in (0, 1):  # stage 2's v by its dyn_tend edge kernel (option vdyn), exact and fast
        for ex in (0, 1):
            c, _ = _two_steps_gpu(st, 1 - vd, ex, 1, vdyn=vd)
            bad = compare_states(c, b if ex == 0 else ref, rtol=0.0)
            assert not bad, f"vdyn={vd}, exact={ex}: {bad[:6]}"
    for d4 in (0, 1):  # rk_step 0's dyn_tend D in stage 1's edge kernel (option defer4), exact and fast
        for ex in (0, 1):
            c, _ = _two_steps_gpu(st, 1 - d4, ex, 1, defer4=d4)
            bad = compare_states(c, b if ex == 0 else ref, rtol=0.0)
            assert not bad, f"defer4={d4}, exact={ex}: {bad[:6]}"
    c, _ = _two_steps_gpu(st, 1, 0, 1, fusesml=0)  # set_smlstep as its own launch
    bad = compare_states(c, b, rtol=0.0)
    assert not bad, f"fusesml=0 vs separate launches: {bad[:6]}"
    for tm in (0, 1):  # dyn_tend's theta_m edge sums (option tmedge) with and without the damping fusion
        c, _ = _two_steps_gpu(st, 1 - tm, 0, 1, tmedge=tm)
        bad = compare_states(c, b, rtol=0.0)
        assert not bad, f"tmedge={tm}, fusedamp={1 - tm} vs separate launches: {bad[:6]}"


def test_fusedamp_dt_zero(x1_2562):
    """dt = 0 (main.rg:66, j = 0): the deferred coefficient is inf; the NaN / inf pattern of
    ru_p is the separate damping's"""
    st = base_state(x1_2562, 5, "ref")
    ref = run_oracle(st, lambda o: o.atm_srk3(0.0, 0))
    got = run_gpu(st, lambda c: T.atm_timestep(c, 0.0), exact=1)
    assert not np.isfinite(ref["ru_p"]).all()
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("L", [56, 63])
@pytest.mark.parametrize("variant", ["random", "mpas0"])
@pytest.mark.parametrize("cve", [1, 4, 8])
def test_dyn_tend_vertex_widths(x1_2562, L, variant, cve):
    """option cve: 1, 4 or 8 vertices per wavefront in dyn_tend's delsq_vorticity, each
    value-identical to the oracle (rk 0, where the del4 terms run)"""
    st = base_state(x1_2562, L, variant)
    ref = run_oracle(st, lambda o: o.atm_compute_dyn_tend_work(0, 720.0))

    def fn(c):
        c.set_option("cve", cve)
        assert c.get_option("cve") == cve
        T.atm_compute_dyn_tend_work(c, 0, 720.0)
    got = run_gpu(st, fn, exact=1)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, f"cve={cve}: {bad[:6]}"
