"""JW baroclinic-wave initial state (mpasdyn/jw.py; init_atm_cases.rg:24-743 in mpas mode,
SURVEY §8.7 row 3).  The reference's init cannot run here and is UB-laden, so the state is
pinned by the properties that define the test case: surface pressure 1000 hPa everywhere,
the discrete hydrostatic balance and equation of state the iteration solves, the 35 m/s
jet, a flat model top at 45 km -- and the reference's own captured behaviour on it: its
RK3 step leaves u and theta_m unchanged (recover_large_step is commented out, Q7)."""
import numpy as np
import pytest

import oracle as O
from mpasdyn import jw
from mpasdyn import mesh as M


@pytest.fixture(scope="module")
def jw26(x1_2562):
    return jw.jw_state(M.zero_based(x1_2562), 26)


def test_vertical_grid():
    g = jw.vertical_grid(26)
    assert np.allclose(g["fzm"][1:26] + g["fzp"][1:26], 1.0, rtol=0, atol=1e-15)
    assert abs(g["cf1"] + g["cf2"] + g["cf3"] - 1.0) < 1e-14
    assert np.all(g["rdzw"][:26] > 0) and g["zw"][26] == pytest.approx(45000.0)


def test_jw_state(jw26):
    st = jw26
    nC, nE, L = st.nCells, st.nEdges, st.L
    assert np.allclose(st["surface_pressure"][:nC, 0], 1.0e5, rtol=1e-12, atol=0)
    g = jw.vertical_grid(L)
    pp, rr = st["pressure_p"][:nC, :L], st["rho_p"][:nC, :L]
    res = pp[:, 1:] - pp[:, :-1] + g["dzu"][1:L] * jw.GRAVITY * (rr[:, :-1] * g["fzp"][1:L] + rr[:, 1:] * g["fzm"][1:L])
    assert np.abs(res).max() < 1e-10 * np.abs(pp).max()
    tt = st["theta_m"][:nC, :L] * st["exner"][:nC, :L]
    eos = rr - (pp / (jw.RGAS * st["zz"][:nC, :L]) - st["rho_base"][:nC, :L] * (tt - jw.T0B)) / tt
    assert np.abs(eos).max() < 1e-12
    u = st["u"][:nE, :L]
    assert 34.0 < np.abs(u).max() <= 35.0
    assert np.allclose(st["zgrid"][:nC, L], 45000.0, rtol=1e-14)
    assert np.all(st["theta_m"][:nC, :L] > 200.0) and np.all(np.diff(st["zgrid"][:nC], axis=1) > 0)
    assert np.allclose(st["rho_zz"][:nC, :L], st["rho_base"][:nC, :L] + rr, rtol=1e-15)
    assert np.abs(st["w"][:nC]).max() < 1e-3  # only the terrain-following slope term


def test_reference_step_keeps_the_state(jw26):
    """the reference's atm_srk3 on the JW state: u and theta_m unchanged (Q7), finite"""
    st = jw26.copy()
    O.Oracle(st).atm_srk3(720.0, 1)
    for f in ("u", "theta_m", "rho_zz"):
        assert np.array_equal(st[f], jw26[f]), f
    assert np.isfinite(st["rtheta_pp"]).all() and np.isfinite(st["rw_p"]).all()


def test_needs_zero_based_mesh(x1_2562):
    from mpasdyn import build_state as bs
    st = bs.build_state(x1_2562, 5, "physical", vertical=False)
    with pytest.raises(ValueError):
        jw.init_atm_case_jw(x1_2562, st)


@pytest.mark.parametrize("L", [2, 3, 26])
def test_hydrostatic_library_matches_numpy(L, monkeypatch):
    """mpas_jw_hydrostatic (host threads in libmpasdyn) and the NumPy statement agree down to
    2 levels (the recurrence reads levels 0 and 1).  Tolerance 1e-14 relative:
    NumPy's vectorised pow/sin may differ from glibc's in the last ulp."""
    from mpasdyn import lib
    rng = np.random.default_rng(7)
    nC = 97
    g = jw.vertical_grid(max(L, 3))
    g = {k: (v[:L + 1] if isinstance(v, np.ndarray) else v) for k, v in g.items()}
    phi = rng.uniform(-1.5, 1.5, nC)
    pb = -np.sort(-rng.uniform(3e4, 1e5, (nC, L)), axis=1)  # eta in (0.3, 1], decreasing upward
    rb = rng.uniform(0.3, 1.2, (nC, L))
    zz = rng.uniform(0.9, 1.1, (nC, L))
    got = jw._hydrostatic(phi, pb, rb, zz, g, L)
    monkeypatch.setattr(lib, "load", lambda: (_ for _ in ()).throw(OSError("numpy path")))
    want = jw._hydrostatic(phi, pb, rb, zz, g, L)
    for a, b in zip(got, want):
        assert np.isfinite(b).all()
        assert np.abs(a - b).max() <= 1e-14 * np.abs(b).max()
