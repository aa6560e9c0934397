"""Mesh ingest, renumbering and partitioning (mpasdyn/meshio.py).

The reference's own grid (x1.2562.grid.nc, carried as tests/golden/x1.2562.mesh.npz) is
written back as a CDF-2 file and read with the product reader; the Morton renumbering is
checked for consistency and, through the oracle, for leaving every mpas-mode result
unchanged up to the permutation (a whole RK3 step, bit-identical); the SFC partitioner
and the part-file format round trip."""
import numpy as np
import pytest

import oracle as O
from mpasdyn import decomp
from mpasdyn import mesh as M
from mpasdyn import meshio

from helpers import compare_states, make_state


def test_grid_roundtrip(tmp_path, x1_2562):
    p = tmp_path / "x1.2562.grid.nc"
    meshio.write_grid(str(p), x1_2562)
    with open(p, "rb") as f:
        assert f.read(4) == b"CDF\x02"  # 64-bit offset format, like the reference's file
    m = meshio.read_grid(str(p))
    assert (m.nCells, m.nEdges, m.nVertices) == (2562, 7680, 5120)
    for v in meshio.GRID_VARS:
        a, b = getattr(m, v), getattr(x1_2562, v)
        assert a.dtype == b.dtype and np.array_equal(a, b), v


def test_grid_missing_variable(tmp_path, x1_2562):
    p = tmp_path / "partial.nc"
    meshio.write_grid(str(p), x1_2562, variables=["latCell", "nEdgesOnCell", "edgesOnCell", "cellsOnEdge",
                                                  "edgesOnEdge", "edgesOnVertex"])
    with pytest.raises(KeyError, match="lonCell"):
        meshio.read_grid(str(p))


def test_renumber_consistent(x1_2562):
    m = x1_2562
    r, perms = meshio.renumber(m)
    for k, n in (("cell", m.nCells), ("edge", m.nEdges), ("vertex", m.nVertices)):
        assert np.array_equal(np.sort(perms[k]), np.arange(n)), k
    pc, pe, pv = perms["cell"], perms["edge"], perms["vertex"]
    assert np.array_equal(r.xCell, m.xCell[pc]) and np.array_equal(r.dvEdge, m.dvEdge[pe])
    assert np.array_equal(r.nEdgesOnCell, m.nEdgesOnCell[pc])
    # new ids resolve to the same old entities, list order kept
    old_of = {"nCells": pc, "nEdges": pe, "nVertices": pv}
    for v, count in M._CONNECTIVITY.items():
        new, old = getattr(r, v), getattr(m, v)[old_of[{"cellsOnCell": "nCells", "edgesOnCell": "nCells",
                                                         "verticesOnCell": "nCells", "cellsOnEdge": "nEdges",
                                                         "verticesOnEdge": "nEdges", "edgesOnEdge": "nEdges",
                                                         "edgesOnVertex": "nVertices",
                                                         "cellsOnVertex": "nVertices"}[v]]]
        n = getattr(m, count)
        ok = (old >= 1) & (old <= n)
        assert np.array_equal(ok, (new >= 1) & (new <= n)), v
        assert np.array_equal(old_of[count][new[ok] - 1] + 1, old[ok]), v
        assert np.array_equal(new[~ok], old[~ok]), v  # padding untouched
    # the file order of x1.2562 is not spatially local; the Morton order is
    def spread(mm):
        c = M.to_zero_based(mm.cellsOnEdge, mm.nCells)
        return float(np.median(np.abs(c[:, 0].astype(np.int64) - c[:, 1])))
    assert spread(r) < spread(m)


def test_renumber_invariance_oracle(x1_2562):
    """mpas-mode ids: the RK3 step of the renumbered state is the renumbered RK3 step"""
    L = 5
    st = make_state(M.zero_based(x1_2562), L, "random")
    _, perms = meshio.renumber(x1_2562)
    sp = meshio.permute_state(st, perms)
    a, b = st.copy(), sp.copy()
    O.Oracle(a).atm_srk3(720.0, 1)
    O.Oracle(b).atm_srk3(720.0, 1)
    bad = compare_states(b, meshio.permute_state(a, perms), rtol=0.0)
    assert not bad, bad[:6]
    # and the permutation is not the identity on anything that matters
    assert not np.array_equal(sp.arrays["cellsOnEdge"], st.arrays["cellsOnEdge"])


def test_permute_state_rejects_ref_ids(x1_2562):
    st = make_state(x1_2562, 5, "ref")
    _, perms = meshio.renumber(x1_2562)
    st.arrays["edgesOnCell"][0, 0] = st.nEdges + 5
    with pytest.raises(ValueError):
        meshio.permute_state(st, perms)


@pytest.mark.parametrize("nparts", [1, 2, 7, 16])
def test_partition_sfc(tmp_path, x1_2562, nparts):
    part = meshio.partition_sfc(x1_2562, nparts)
    counts = np.bincount(part, minlength=nparts)
    assert counts.sum() == x1_2562.nCells and counts.max() - counts.min() <= 1
    p = tmp_path / f"x1.2562.graph.info.part.{nparts}"
    meshio.write_graph_info_part(str(p), part)
    assert np.array_equal(meshio.read_graph_info_part(str(p), x1_2562.nCells), part)


def test_partition_sfc_interior(x1_2562):
    """renumbered + SFC-partitioned x1.2562 / 4: most owned cells are interior (reach no
    ghost), the overlap's lever; the file order of the mesh has none"""
    r = M.zero_based(meshio.renumber(x1_2562)[0])  # (renumber reads the file's 1-based ids)
    st = make_state(r, 5, "random")
    part = meshio.partition_sfc(r, 4)
    dec = decomp.Decomposition(st, 4, cell_part=part)
    for rank in range(4):
        nint, own = dec.n_interior(rank)[0], dec.n_owned(rank)[0]
        assert nint / own > 0.5, (rank, nint, own)


def test_partition_sfc_bad():
    m = M.Mesh(nEdgesOnCell=np.zeros(3, np.int32), cellsOnEdge=np.zeros((2, 2), np.int32),
               edgesOnVertex=np.zeros((1, 3), np.int32), xCell=np.zeros(3), yCell=np.zeros(3), zCell=np.zeros(3))
    with pytest.raises(ValueError):
        meshio.partition_sfc(m, 4)


def test_meshio_cli(tmp_path, x1_2562):
    g = tmp_path / "x1.2562.grid.nc"
    meshio.write_grid(str(g), x1_2562)
    out = tmp_path / "x1.2562.morton.grid.nc"
    meshio.main([str(g), "--renumber", str(out), "--parts", "8"])
    r = meshio.read_grid(str(out))
    assert np.array_equal(r.xCell, meshio.renumber(x1_2562)[0].xCell)
    part = meshio.read_graph_info_part(str(tmp_path / "x1.2562.morton.graph.info.part.8"), r.nCells)
    assert np.array_equal(part, meshio.partition_sfc(r, 8))


def test_write_output_plotting(tmp_path, x1_2562):
    """mesh_loading.rg:810-1191: grid variables + level 0 of the output fields, after
    atm_compute_output_diagnostics (oracle)"""
    from scipy.io import netcdf_file
    st = make_state(x1_2562, 5, "random")
    O.Oracle(st).atm_compute_output_diagnostics()
    p = tmp_path / "timestep_output.nc"
    meshio.write_output_plotting(str(p), x1_2562, st)
    with netcdf_file(str(p), "r", mmap=False) as f:
        assert f.dimensions["nVertLevels"] == 5 and f.dimensions["Time"] is None
        assert np.array_equal(f.variables["edgesOnCell"].data, x1_2562.edgesOnCell)
        assert np.array_equal(f.variables["indexToEdgeID"].data, np.arange(1, x1_2562.nEdges + 1))
        assert np.array_equal(f.variables["u"].data, st["u"][:x1_2562.nEdges, 0])
        assert np.array_equal(f.variables["rho"].data, st["rho_zz"][:2562, 0] * st["zz"][:2562, 0])
        assert np.array_equal(f.variables["pressure"].data, st["pressure"][:2562, 0])
        assert "dv1Edge" not in f.variables  # not in the grid fixture
