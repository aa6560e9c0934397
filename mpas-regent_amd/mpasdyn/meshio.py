"""Mesh ingest, renumbering and partitioning.

* ``read_grid(path)`` -- an MPAS grid file (netCDF classic / CDF-2 64-bit offset, the
  format of the reference's ``mesh_loading/x1.2562.grid.nc``), the variables the
  reference reads in ``mesh_loading.rg:123-201``, as a ``mesh.Mesh`` with the file's
  1-based ids and its unit-sphere distances (``init_atm_cases.rg:87-111`` scales by the
  sphere radius later, in the state builder).  ``write_grid`` writes the same subset.
* ``renumber(m)`` -- cells, edges and vertices each sorted along a space-filling curve
  (cube-face 2-D Hilbert by default, ``order="morton"`` the 3-D Morton key) of
  their (x, y, z) position, connectivity remapped; the order of every connectivity list
  is kept, so in mpas-mode (0-based) ids every per-entity result is unchanged and only
  its position moves.  Neighbour gathers then stay close in HBM, and a contiguous
  partition has few boundary entities (the overlap's interior share).
  (The reference's "ref" mode uses raw 1-based ids as offsets -- SURVEY Q1 -- which a
  renumbering changes; renumber before building a "ref" state only on purpose.)
* ``partition_sfc(m, nparts)`` -- balanced contiguous blocks of cells along the same
  curve, the build's partitioner for meshes without a METIS part file;
  ``read_graph_info_part`` / ``write_graph_info_part`` -- the part-file format of
  ``mesh_loading.rg:11-22`` (one 0-based part id per line).

Host-side NumPy/SciPy: no GPU work, nothing here is on the timed path.
"""
import numpy as np

from . import mesh as M

# the grid variables of mesh_loading.rg:123-201 (the reference's x1 grid files)
GRID_VARS = ["latCell", "lonCell", "xCell", "yCell", "zCell", "meshDensity", "areaCell",
             "nEdgesOnCell", "edgesOnCell", "cellsOnCell", "verticesOnCell",
             "latEdge", "lonEdge", "xEdge", "yEdge", "zEdge", "cellsOnEdge", "verticesOnEdge",
             "nEdgesOnEdge", "edgesOnEdge", "weightsOnEdge", "dvEdge", "dcEdge", "angleEdge",
             "latVertex", "lonVertex", "xVertex", "yVertex", "zVertex", "areaTriangle",
             "edgesOnVertex", "cellsOnVertex", "kiteAreasOnVertex"]

# netCDF dimension names of each variable (MPAS grid convention)
_DIMS = {"nEdgesOnCell": ("nCells",), "edgesOnCell": ("nCells", "maxEdges"),
         "cellsOnCell": ("nCells", "maxEdges"), "verticesOnCell": ("nCells", "maxEdges"),
         "cellsOnEdge": ("nEdges", "TWO"), "verticesOnEdge": ("nEdges", "TWO"),
         "nEdgesOnEdge": ("nEdges",), "edgesOnEdge": ("nEdges", "maxEdges2"),
         "weightsOnEdge": ("nEdges", "maxEdges2"), "edgesOnVertex": ("nVertices", "vertexDegree"),
         "cellsOnVertex": ("nVertices", "vertexDegree"), "kiteAreasOnVertex": ("nVertices", "vertexDegree")}
for _v in GRID_VARS:
    if _v not in _DIMS:
        _DIMS[_v] = ("nCells",) if _v.endswith("Cell") or _v in ("meshDensity",) else \
            ("nEdges",) if _v.endswith("Edge") else ("nVertices",)
_DIMS["areaTriangle"] = ("nVertices",)


def read_grid(path, variables=GRID_VARS):
    """An MPAS grid file as a Mesh (ids 1-based as stored; integer arrays int32, real
    arrays float64).  Raises KeyError naming a missing variable."""
    from scipy.io import netcdf_file
    with netcdf_file(path, "r", mmap=False) as f:
        out = {}
        for v in variables:
            if v not in f.variables:
                raise KeyError(f"{path}: grid variable {v!r} missing")
            a = np.asarray(f.variables[v].data)
            out[v] = np.ascontiguousarray(a.astype(np.int32 if a.dtype.kind in "iu" else np.float64))
    return M.Mesh(**out)


def write_grid(path, m, variables=GRID_VARS):
    """Write the grid variables of m as a CDF-2 (64-bit offset) netCDF file."""
    from scipy.io import netcdf_file
    dims = {"nCells": m.nCells, "nEdges": m.nEdges, "nVertices": m.nVertices, "TWO": 2,
            "maxEdges": m.edgesOnCell.shape[1], "maxEdges2": m.edgesOnEdge.shape[1],
            "vertexDegree": m.edgesOnVertex.shape[1]}
    with netcdf_file(path, "w", version=2) as f:
        for d, n in dims.items():
            f.createDimension(d, int(n))
        for v in variables:
            a = np.asarray(getattr(m, v))
            var = f.createVariable(v, "i4" if a.dtype.kind in "iu" else "f8", _DIMS[v])
            var[:] = a


def _curve_order(x, y, z, order="hilbert"):
    """permutation sorting the points along a space-filling curve (mesh._order_key: "hilbert",
    2-D Hilbert curves on the cube faces, or "morton", the 3-D Morton key)"""
    p = np.stack([x, y, z], axis=1).astype(np.float64)
    if order == "hilbert":  # direction only: the cube-face projection needs no radius
        p = p / np.maximum(np.linalg.norm(p, axis=1), 1e-300)[:, None]
    else:
        p = p / max(float(np.abs(p).max()), 1e-300)  # any sphere radius -> [-1, 1]
    return np.argsort(M._order_key(p, order), kind="stable")


def _remap(ids, new_of_old, n):
    """1-based ids through a permutation (old 0-based -> new 0-based); values outside
    1..n (file padding) are kept as stored"""
    ids = np.asarray(ids)
    out = ids.copy()
    ok = (ids >= 1) & (ids <= n)
    out[ok] = new_of_old[ids[ok] - 1] + 1
    return out.astype(ids.dtype)


_ROWS = {"nCells": ["latCell", "lonCell", "xCell", "yCell", "zCell", "meshDensity", "areaCell", "nEdgesOnCell",
                    "edgesOnCell", "cellsOnCell", "verticesOnCell"],
         "nEdges": ["latEdge", "lonEdge", "xEdge", "yEdge", "zEdge", "cellsOnEdge", "verticesOnEdge", "nEdgesOnEdge",
                    "edgesOnEdge", "weightsOnEdge", "dvEdge", "dcEdge", "angleEdge"],
         "nVertices": ["latVertex", "lonVertex", "xVertex", "yVertex", "zVertex", "areaTriangle", "edgesOnVertex",
                       "cellsOnVertex", "kiteAreasOnVertex"]}


def renumber(m, order="hilbert"):
    """(renumbered Mesh, {"cell": old_of_new, "edge": ..., "vertex": ...}): each entity
    kind sorted along a space-filling curve of its position (order "hilbert": 2-D Hilbert
    curves on the faces of the circumscribed cube; "morton": the 3-D Morton key); a new entity i is old entity
    old_of_new[i].  Row order of every per-entity array and the values of every
    connectivity array follow; the order inside each connectivity list is kept.  m holds
    the file's 1-based ids (read_grid, mesh.icosahedral); convert with mesh.zero_based
    afterwards for mpas mode."""
    perm = {"nCells": _curve_order(m.xCell, m.yCell, m.zCell, order),
            "nEdges": _curve_order(m.xEdge, m.yEdge, m.zEdge, order),
            "nVertices": _curve_order(m.xVertex, m.yVertex, m.zVertex, order)}
    new_of_old = {}
    for k, p in perm.items():
        inv = np.empty_like(p)
        inv[p] = np.arange(p.size)
        new_of_old[k] = inv
    d = {}
    for count, names in _ROWS.items():
        for v in names:
            if hasattr(m, v):
                d[v] = np.ascontiguousarray(np.asarray(getattr(m, v))[perm[count]])
    for v, count in M._CONNECTIVITY.items():
        if v in d:
            d[v] = _remap(d[v], new_of_old[count], getattr(m, count))
    for v, a in m.__dict__.items():  # anything else (e.g. a part array) rides along unchanged
        if v not in d and v not in ("nCells", "nEdges", "nVertices"):
            d[v] = a
    if hasattr(m, "part"):
        d["part"] = np.asarray(m.part)[perm["nCells"]]
    out = M.Mesh(**d)
    return out, {"cell": perm["nCells"], "edge": perm["nEdges"], "vertex": perm["nVertices"]}


# the state's integer fields that hold entity ids, and the kind they refer to
ID_FIELDS = {"edgesOnCell": "edge", "verticesOnCell": "vertex", "cellsOnEdge": "cell", "verticesOnEdge": "vertex",
             "edgesOnEdge": "edge", "edgesOnEdge_ECP": "edge", "advCellsForEdge": "cell", "edgesOnVertex": "edge",
             "cellsOnCell": "cell", "cellsOnVertex": "cell"}


def permute_state(st, perms):
    """A copy of a state with mpas-mode (0-based, zero slot n) ids, renumbered by the
    permutations of renumber(): every per-entity row moves to its new position (the zero
    slot stays last) and every id field is remapped.  The hot path's result for the
    permuted state is the permutation of its result for st (tests/test_meshio.py)."""
    from .registry import FIELDS
    n = {"cell": st.nCells, "edge": st.nEdges, "vertex": st.nVertices}
    new_of_old = {}
    for k, p in perms.items():
        inv = np.empty(p.size + 1, dtype=np.int64)
        inv[p] = np.arange(p.size)
        inv[p.size] = p.size  # zero slot
        new_of_old[k] = inv
    out = st.copy()
    for f in FIELDS:
        ent = f.entity
        if ent is None:
            continue
        a = st.arrays[f.name]
        b = a.copy()
        b[: n[ent]] = a[perms[ent]]
        if f.name in ID_FIELDS:
            tgt = ID_FIELDS[f.name]
            ids = b.astype(np.int64)
            if ids.min() < 0 or ids.max() > n[tgt]:
                raise ValueError(f"{f.name}: ids outside [0, {n[tgt]}] (not an mpas-mode state?)")
            b = new_of_old[tgt][ids].astype(a.dtype)
        out.arrays[f.name] = b
    return out


def partition_sfc(m, nparts, order="hilbert"):
    """0-based part id per cell: nparts contiguous, balanced (sizes differ by <= 1)
    blocks of cells along a space-filling curve of their positions (renumber's orders)."""
    if nparts < 1 or nparts > m.nCells:
        raise ValueError(f"nparts={nparts} for {m.nCells} cells")
    order = _curve_order(m.xCell, m.yCell, m.zCell, order)
    part = np.empty(m.nCells, dtype=np.int32)
    bounds = np.linspace(0, m.nCells, nparts + 1).round().astype(np.int64)
    for p in range(nparts):
        part[order[bounds[p]:bounds[p + 1]]] = p
    return part


def read_graph_info_part(path, nCells):
    """mesh_loading.rg:11-22: one 0-based part id per line, one line per cell"""
    return M.read_graph_info_part(path, nCells)


def write_graph_info_part(path, part):
    """the same format, one id per line"""
    np.savetxt(path, np.asarray(part, dtype=np.int64), fmt="%d")


# write_output_plotting (mesh_loading.rg:810-1191): the mesh variables it defines (those
# the Mesh holds), then level 0 of the state fields below
OUTPUT_MESH_VARS = ["latCell", "lonCell", "meshDensity", "xCell", "yCell", "zCell", "latEdge", "lonEdge",
                    "xEdge", "yEdge", "zEdge", "latVertex", "lonVertex", "xVertex", "yVertex", "zVertex",
                    "cellsOnEdge", "nEdgesOnCell", "nEdgesOnEdge", "edgesOnCell", "edgesOnEdge", "weightsOnEdge",
                    "dvEdge", "dv1Edge", "dv2Edge", "dcEdge", "angleEdge", "areaCell", "areaTriangle", "cellsOnCell",
                    "verticesOnCell", "verticesOnEdge", "edgesOnVertex", "cellsOnVertex", "kiteAreasOnVertex"]
OUTPUT_STATE_VARS = {"u": "nEdges", "v": "nEdges", "w": "nCells", "pressure": "nCells", "pressure_p": "nCells",
                     "rho": "nCells", "theta": "nCells", "surface_pressure": "nCells"}


def write_output_plotting(path, m, st):
    """timestep_output.nc as mesh_loading.rg:810-1191 writes it: the grid variables,
    indexToCellID/EdgeID/VertexID (1-based), and level 0 of u, v (edges), w, pressure,
    pressure_p, rho, theta, surface_pressure (cells) from the state st (e.g. after
    atm_compute_output_diagnostics and a download).  Grid variables the Mesh does not
    hold (dv1Edge, dv2Edge for the generated meshes) are left out."""
    from scipy.io import netcdf_file
    dims = {"nCells": m.nCells, "nEdges": m.nEdges, "nVertices": m.nVertices,
            "maxEdges": m.edgesOnCell.shape[1], "maxEdges2": m.edgesOnEdge.shape[1], "TWO": 2,
            "vertexDegree": m.edgesOnVertex.shape[1], "nVertLevels": st.L}
    with netcdf_file(path, "w", version=2) as f:
        f.createDimension("Time", None)  # (scipy's writer wants the record dimension first)
        for d, n in dims.items():
            f.createDimension(d, int(n))
        for v in OUTPUT_MESH_VARS:
            if not hasattr(m, v):
                continue
            a = np.asarray(getattr(m, v))
            dv = _DIMS.get(v, ("nEdges",))
            var = f.createVariable(v, "i4" if a.dtype.kind in "iu" else "f8", dv)
            var[:] = a
        for v, n in (("indexToCellID", m.nCells), ("indexToEdgeID", m.nEdges), ("indexToVertexID", m.nVertices)):
            f.createVariable(v, "i4", ({"indexToCellID": "nCells", "indexToEdgeID": "nEdges"}.get(v, "nVertices"),))[:] = \
                np.arange(1, n + 1, dtype=np.int32)
        for v, dim in OUTPUT_STATE_VARS.items():
            n = dims[dim]
            f.createVariable(v, "f8", (dim,))[:] = np.asarray(st[v])[:n, 0]


def main(argv=None):
    """python -m mpasdyn.meshio GRID.nc [--renumber OUT.nc] [--parts N] [--order hilbert|morton]: read an MPAS grid,
    optionally write it renumbered along the curve, optionally write OUT's (or GRID's)
    graph.info.part.N from the SFC partitioner."""
    import argparse
    ap = argparse.ArgumentParser(prog="python -m mpasdyn.meshio")
    ap.add_argument("grid")
    ap.add_argument("--renumber", metavar="OUT.nc")
    ap.add_argument("--parts", type=int, default=0)
    ap.add_argument("--order", choices=["hilbert", "morton"], default="hilbert")
    a = ap.parse_args(argv)
    m = read_grid(a.grid)
    base = a.grid
    if a.renumber:
        m, _ = renumber(m, a.order)
        write_grid(a.renumber, m)
        base = a.renumber
    if a.parts:
        stem = base[:-3] if base.endswith(".nc") else base
        stem = stem[:-5] if stem.endswith(".grid") else stem
        write_graph_info_part(f"{stem}.graph.info.part.{a.parts}", partition_sfc(m, a.parts, a.order))
    print(f"{a.grid}: nCells={m.nCells} nEdges={m.nEdges} nVertices={m.nVertices}")


if __name__ == "__main__":
    main()
