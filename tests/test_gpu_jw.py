"""The JW initial state on the GPU: RK3 steps from it match the oracle bit for bit (exact
mode), and the end-to-end driver (mpasdyn/driver.py, main.rg's loop) writes
timestep_output.nc."""
import numpy as np
import pytest

import oracle as O
from helpers import ZERO_SLOT_WRITTEN, compare_states
from mpasdyn import jw, lib
from mpasdyn import mesh as M
from mpasdyn import tasks as T

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("L", [5, 26, 56])  # (5: the reference's default, constants.rg:26, BASELINE config 1)
def test_jw_steps_match_oracle(x1_2562, L):
    st = jw.jw_state(M.zero_based(x1_2562), L)
    ref = st.copy()
    o = O.Oracle(ref)
    for _ in range(2):
        o.atm_srk3(720.0, 1)
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", 1)
        ctx.upload(st)
        for _ in range(2):
            T.atm_srk3(ctx, 720.0, 1)
        ctx.sync()
        ctx.download(got)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("schedule", [0, 1])
def test_jw_config1_fast_path(x1_2562, schedule):
    """BASELINE config 1 (x1.2562 x 5 levels) from the JW state on the benchmark path (exact 0, graph
    replay): within the fast path's step tolerance of the oracle, NaN / inf masks equal, for the
    reference's driver schedule (0) and the MPAS one (1)"""
    st = jw.jw_state(M.zero_based(x1_2562), 5)
    ref = st.copy()
    o = O.Oracle(ref)
    for _ in range(3):
        o.atm_srk3(720.0, schedule)
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", 0)
        ctx.upload(st)
        for _ in range(3):
            T.atm_srk3(ctx, 720.0, schedule)
        ctx.sync()
        ctx.download(got)
    bad = compare_states(got, ref, rtol=1e-9)
    assert not bad, bad[:6]


@pytest.mark.parametrize("physics", [1, 2])
def test_jw_config1_mpas(x1_2562, physics):
    """the MPAS solver / dynamics from the JW state at 5 levels: exact mode = the oracle bit for bit but
    for the pow of recover's exner / pressure_p (device pow against glibc's: 1e-14)"""
    st = jw.jw_state(M.zero_based(x1_2562), 5)
    ref = st.copy()
    O.Oracle(ref).mpas_srk3(720.0, 1, physics=physics)
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", 1)
        ctx.set_option("physics", physics)
        ctx.upload(st)
        T.atm_srk3(ctx, 720.0, 1)
        ctx.sync()
        ctx.download(got)
    bad = compare_states(got, ref, rtol=1e-14, tol_fields={"exner", "pressure_p"}, zero_slot_excluded=ZERO_SLOT_WRITTEN)
    assert not bad, bad[:6]


def test_driver_end_to_end(x1_2562, tmp_path):
    from scipy.io import netcdf_file
    from mpasdyn import driver
    out = str(tmp_path / "timestep_output.nc")
    lines = []
    st = driver.run(x1_2562, 26, 3, 720.0, out=out, log=lines.append)
    assert len(lines) == 3
    with netcdf_file(out, "r", mmap=False) as f:
        sp = f.variables["surface_pressure"][:].copy()
        u = f.variables["u"][:].copy()
        rho = f.variables["rho"][:].copy()
    assert np.allclose(sp, 1.0e5, rtol=1e-12)
    assert np.array_equal(u, st["u"][:st.nEdges, 0])  # level 0 (the jet peaks aloft)
    assert 34.0 < np.abs(st["u"][:st.nEdges, :26]).max() <= 35.0  # u unchanged by the steps (Q7)
    assert np.allclose(rho, st["rho_zz"][:st.nCells, 0] * st["zz"][:st.nCells, 0], rtol=1e-15)


def test_core_init_keeps_jw_terrain_coefficients(x1_2562):
    """main.rg:57-61 order: the JW state (with its terrain-slope zb_cell / zb3_cell, the copy
    of er.zb that init_atm_case_jw writes, init_atm_cases.rg:657-660) is uploaded, then
    atm_core_init runs: atm_compute_signs must not erase zb_cell, and only
    atm_couple_coef_3rd_order scales zb3_cell at level 0 (:319-323)"""
    st = jw.jw_state(M.zero_based(x1_2562), 26)
    nC = st.nCells
    assert np.abs(st["zb_cell"][:nC]).max() > 0.0
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.upload(st)
        T.atm_compute_signs(ctx)
        ctx.sync()
        ctx.download(got, names=["zb_cell", "zb3_cell"])
        assert np.array_equal(got["zb_cell"], st["zb_cell"]) and np.array_equal(got["zb3_cell"], st["zb3_cell"])
        T.atm_core_init(ctx)
        ctx.sync()
        ctx.download(got, names=["zb_cell", "zb3_cell"])
    assert np.array_equal(got["zb_cell"], st["zb_cell"])
    assert np.array_equal(got["zb3_cell"][:, 1:], st["zb3_cell"][:, 1:])
    ref = st.copy()
    O.Oracle(ref).atm_couple_coef_3rd_order(0.25)
    assert np.array_equal(got["zb3_cell"][:nC, 0], ref["zb3_cell"][:nC, 0])
