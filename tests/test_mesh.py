"""Mesh fixture and the icosahedral x1.N generator."""
import numpy as np
import pytest

from mpasdyn import mesh
from mpasdyn.state import HostState


def test_fixture_counts(x1_2562):
    m = x1_2562
    assert (m.nCells, m.nEdges, m.nVertices) == (2562, 7680, 5120)  # constants.rg:18-20
    assert m.part.shape == (2562,) and m.part.min() == 0 and m.part.max() == 15
    assert m.cellsOnEdge.min() == 1 and m.cellsOnEdge.max() == 2562  # 1-based file ids (Q1)


@pytest.mark.parametrize("level", [2, 4, 5])
@pytest.mark.parametrize("order", ["hilbert", "morton"])
def test_icosahedral_topology(level, order):
    m = mesh.icosahedral(level, order=order)
    n = 10 * 4 ** level + 2
    assert (m.nCells, m.nEdges, m.nVertices) == (n, 3 * (n - 2), 2 * (n - 2))
    assert sorted(set(m.nEdgesOnCell.tolist())) == [5, 6]
    assert (m.nEdgesOnCell == 5).sum() == 12
    c = np.arange(m.nCells)
    for j in range(6):
        e = m.edgesOnCell[:, j] - 1
        on = (m.cellsOnEdge[e, 0] - 1 == c) | (m.cellsOnEdge[e, 1] - 1 == c)
        assert (on | (j >= m.nEdgesOnCell)).all()
    # every edge appears in the edge list of both its cells
    cnt = np.zeros(m.nEdges, int)
    for j in range(6):
        np.add.at(cnt, m.edgesOnCell[:, j][j < m.nEdgesOnCell] - 1, 1)
    assert (cnt == 2).all()
    # vertices: both cells of each vertex edge belong to the vertex
    for j in range(3):
        e = m.edgesOnVertex[:, j] - 1
        for s in range(2):
            assert ((m.cellsOnVertex - 1) == (m.cellsOnEdge[e, s] - 1)[:, None]).any(1).all()
    assert (m.nEdgesOnEdge == m.nEdgesOnCell[m.cellsOnEdge[:, 0] - 1] + m.nEdgesOnCell[m.cellsOnEdge[:, 1] - 1] - 2).all()


@pytest.mark.parametrize("level", [3, 4])
def test_icosahedral_geometry(level):
    m = mesh.icosahedral(level)
    assert abs(m.areaCell.sum() - 4 * np.pi) < 1e-9
    assert abs(m.areaTriangle.sum() - 4 * np.pi) < 1e-9
    assert abs(m.kiteAreasOnVertex.sum() - 4 * np.pi) < 1e-9
    # the same scales as the reference's own x1.2562 grid (unit sphere)
    if level == 4:
        f = mesh.load_x1_2562()
        for k in ("dcEdge", "dvEdge", "areaCell"):
            assert 0.8 < np.median(getattr(m, k)) / np.median(getattr(f, k)) < 1.25


def test_curve_orders_locality():
    """both numberings keep neighbouring cells close; the cube-face Hilbert curve (the
    default) more often than the 3-D Morton key"""
    far = {}
    for order in ("hilbert", "morton"):
        m = mesh.icosahedral(5, order=order)
        c = m.cellsOnEdge - 1
        d = np.abs(c[:, 0] - c[:, 1])
        assert np.median(d) <= 8
        far[order] = (d > 64).mean()
    assert far["hilbert"] < far["morton"]
    with pytest.raises(ValueError):
        mesh.icosahedral(1, order="peano")


def test_zero_based_conversion():
    ids = np.array([[1, 2, 0], [3, 0, 0]], np.int32)
    assert mesh.to_zero_based(ids, 3).tolist() == [[0, 1, 3], [2, 3, 3]]


def test_hoststate_layout():
    st = HostState(4, 9, 6, 5)
    assert st["theta_m"].shape == (5, 6)
    assert st["zb_cell"].shape == (5, 6, 10)
    assert st["edgesOnCell"].shape == (5, 10)
    assert st["rdzw"].shape == (6,)
    se, sl, sc = st.byte_strides("zb_cell")
    assert (se, sl, sc) == (6 * 10 * 8, 10 * 8, 8)
