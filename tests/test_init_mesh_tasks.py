"""The mesh tasks of atm_core_init (atm_core.rg:22-39) in the oracle against the host
restatements of mpasdyn/build_state.py that build every test and benchmark state:
atm_compute_signs (dynamics_tasks.rg:46-130), atm_adv_coef_compression (:133-269) with
atm_couple_coef_3rd_order (:303-325), atm_compute_mesh_scaling (:595-646).  Both follow the
reference's raw ids (Q1): the 1-based ids of the reference's x1.2562 mesh ("ref") and the
0-based ones of mpas mode.  Bit-identical except meshScalingDel2/4 (pow of libm vs NumPy)."""
import numpy as np
import pytest

import oracle as O
from mpasdyn import build_state as bs
from mpasdyn import mesh as M

L = 5
DERIVED = ["edgesOnVertexSign", "edgesOnCellSign", "kiteForCell", "nAdvCellsForEdge", "advCellsForEdge",
           "adv_coefs", "adv_coefs_3rd"]


def _state(x1_2562, ids):
    m = x1_2562 if ids == "raw" else M.zero_based(x1_2562)
    return m, bs.build_state(m, L, "ref")


@pytest.mark.parametrize("ids", ["raw", "zero_based"])
def test_mesh_tasks_match_build_state(x1_2562, ids):
    m, st = _state(x1_2562, ids)
    got = st.copy()
    for f in DERIVED + ["meshScalingDel2", "meshScalingDel4"]:
        got[f][...] = 0
    o = O.Oracle(got)
    o.atm_compute_signs()
    o.atm_adv_coef_compression()
    o.atm_couple_coef_3rd_order(0.25)
    o.atm_compute_mesh_scaling(True)
    for f in DERIVED:
        a, b = got[f], st[f]
        assert a.shape == b.shape
        assert np.array_equal(a, b, equal_nan=True), f
        assert np.array_equal(np.signbit(a), np.signbit(b)), f  # -0.0 of the coefficient loop
    for f in ("meshScalingDel2", "meshScalingDel4"):
        assert np.allclose(got[f], st[f], rtol=1e-15, atol=0), f
    # the tasks did something: the lists, signs and the 2nd-order weights
    nE = st.nEdges
    n = got["nAdvCellsForEdge"][:nE, 0]
    assert n.min() >= 6 and (n == 9).mean() > 0.99
    assert np.isclose(got["adv_coefs"][:nE].sum(axis=1), got["dvEdge"][:nE, 0]).all()


def test_mesh_tasks_quirks(x1_2562):
    """the literal list construction: nAdvCellsForEdge = n is the index of the last cell
    (:184), so that cell is never weighted; deriv_two (never initialised, Q2) feeds the
    3rd/4th-order weights when given; zb_cell / zb3_cell (the copy of er.zb that
    init_atm_case_jw writes, init_atm_cases.rg:657-660, done by the host that uploads them)
    stay as given -- only couple_coef_3rd_order scales zb3_cell at level 0"""
    m, st = _state(x1_2562, "zero_based")
    nE, nC = st.nEdges, st.nCells
    st["deriv_two"][:nE] = np.random.default_rng(3).standard_normal((nE, 30))
    st["zb_cell"][:nC] = 1.0
    st["zb3_cell"][:nC] = 1.0
    ref = st.copy()
    bs.adv_coef_compression_loops(m, ref, st["dcEdge"][:nE, 0], st["dvEdge"][:nE, 0], deriv_two=st["deriv_two"][:nE])
    o = O.Oracle(st)
    o.atm_compute_signs()
    o.atm_adv_coef_compression()
    o.atm_couple_coef_3rd_order(0.25)
    for f in ("adv_coefs", "adv_coefs_3rd", "advCellsForEdge", "nAdvCellsForEdge"):
        assert np.array_equal(st[f], ref[f]), f
    n = st["nAdvCellsForEdge"][:nE, 0]
    # only entries 0..n-1 are stored (:185-187): the list's last cell is dropped
    assert (st["advCellsForEdge"][np.arange(nE), n] == 0).all()
    ne = st["nEdgesOnCell"][:nC, 0]
    assert (st["zb_cell"][:nC] == 1.0).all()  # as uploaded
    # couple_coef_3rd_order scales zb3_cell at level 0 only (:319-323)
    assert (st["zb3_cell"][:nC, 1:] == 1.0).all()
    assert (st["zb3_cell"][:nC, 0] == 0.25).all()
