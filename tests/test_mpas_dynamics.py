"""The MPAS dynamics (option physics = 2; oracle ora_mpas_* in oracle/mpas_oracle.c) on the
CPU: with every quirk of the path fixed the split-explicit RK3 step is a dynamical core,
so the JW test case's defining behaviour pins the oracle (PARITY UNPINNED against the
reference, which never changes its state, Q7).  The unperturbed JW state is a steady
solution of the dry primitive equations: over one simulated day (x1.2562, 26 levels,
720 s steps) it must stay balanced -- surface pressure within 1 hPa of its initial
1000 hPa, vertical velocity small, the jet within a few m/s -- with the dry mass
sum(rho_zz volume) conserved to round-off (flux form).  A localised zonal-wind
perturbation must instead grow the baroclinic wave: the dynamics is not frozen
(measured: the perturbed-minus-balanced surface pressure grows from 0.3 hPa at day 1 to
2.0 at day 5 and 46 at day 9; surface pressure 955-1023 hPa at day 9)."""
import numpy as np
import pytest

import oracle as O
from mpasdyn import jw
from mpasdyn import mesh as M

L = 26
DT = 720.0


def jw_oracle(x1_2562, perturb=False):
    st = jw.jw_state(M.zero_based(x1_2562), L, perturb=perturb)
    o = O.Oracle(st)
    o.mpas_solve_diagnostics(0, -1)  # MPAS-A's initial diagnostics (atm_core_init)
    o.mpas_reconstruct_2d(False, True)
    return st, o


def volumes(st):
    nC = st.nCells
    return 1.0 / (st["invAreaCell"][:nC, 0][:, None] * st["rdzw"][:L][None, :])


def test_jw_balanced_for_a_day(x1_2562):
    st, o = jw_oracle(x1_2562)
    nC, nE = st.nCells, st.nEdges
    vol = volumes(st)
    o.mpas_surface_pressure()
    sp0 = st["surface_pressure"][:nC, 0].copy()
    u0 = st["u"][:nE, :L].copy()
    mass0 = np.sum(st["rho_zz"][:nC, :L] * vol)
    assert np.allclose(sp0, 1.0e5, rtol=1e-12)
    for _ in range(int(86400 / DT)):
        o.mpas_srk3(DT, 1, physics=2)
    o.mpas_surface_pressure()
    sp = st["surface_pressure"][:nC, 0]
    assert np.isfinite(st["u"][:nE, :L]).all() and np.isfinite(st["w"][:nC, :L + 1]).all()
    assert np.abs(sp - 1.0e5).max() < 100.0  # within 1 hPa after a day
    assert np.abs(st["w"][:nC, :L + 1]).max() < 0.05
    assert np.abs(st["u"][:nE, :L] - u0).max() < 5.0
    mass = np.sum(st["rho_zz"][:nC, :L] * vol)
    assert abs(mass / mass0 - 1.0) < 1e-12
    # the step is not the identity: the state moved
    assert np.abs(sp - sp0).max() > 1.0 and np.abs(st["u"][:nE, :L] - u0).max() > 0.1


def test_jw_perturbation_grows_a_wave(x1_2562):
    """the JW test's u perturbation (1 m/s, centred at 20E 40N): after a day the surface
    pressure departs from the balanced run's mainly in the northern mid-latitudes (the
    adjustment's gravity waves reach the south weakly); by day 6 the baroclinic wave has
    grown to several hPa (the balanced run stays within 1 hPa); mass is conserved"""
    st, o = jw_oracle(x1_2562, perturb=True)
    stb, ob = jw_oracle(x1_2562)
    vol = volumes(st)
    nC = st.nCells
    mass0 = np.sum(st["rho_zz"][:nC, :L] * vol)
    lat = st["lat"][:nC, 0]
    for day in range(1, 7):
        for _ in range(int(86400 / DT)):
            o.mpas_srk3(DT, 1, physics=2)
            if day == 1:
                ob.mpas_srk3(DT, 1, physics=2)
        if day == 1:
            o.mpas_surface_pressure()
            ob.mpas_surface_pressure()
            d = st["surface_pressure"][:nC, 0] - stb["surface_pressure"][:nC, 0]
            assert np.isfinite(d).all() and np.abs(d).max() > 1.0  # the perturbation propagates
            i = np.argmax(np.abs(d))
            assert 0.5 < lat[i] < 1.2  # ... from the northern mid-latitudes
            assert np.abs(d[lat < 0]).max() < 0.5 * np.abs(d[lat > 0]).max()
    o.mpas_surface_pressure()
    sp = st["surface_pressure"][:nC, 0]
    assert np.isfinite(sp).all() and sp.max() - sp.min() > 500.0  # > 5 hPa: the wave grew
    assert abs(np.sum(st["rho_zz"][:nC, :L] * vol) / mass0 - 1.0) < 1e-12


def test_mpas_dyn_tend_keeps_state_w(x1_2562):
    """Q8 fixed: the MPAS dyn_tend writes its w tendency to tend_w and leaves the state w
    and every field it does not own untouched"""
    st, o = jw_oracle(x1_2562)
    before = st.copy()
    o.mpas_rk_integration_setup()
    o.mpas_dyn_tend(0, DT)
    assert np.array_equal(st["w"], before["w"])
    assert np.any(st["tend_w"][:st.nCells, 1:L] != 0.0)
    assert np.all(st["tend_w"][:st.nCells, 0] == 0.0) and np.all(st["tend_w"][:st.nCells, L] == 0.0)
