"""Meshes for the RK3 hot path.

* ``load_x1_2562()`` -- the reference's own mesh (mesh_loading/x1.2562.grid.nc, converted
  verbatim to tests/golden/x1.2562.mesh.npz) and its METIS partition
  x1.2562.graph.info.part.16, read like mesh_loading.rg:11-22.
* ``icosahedral(level)`` -- x1.N quasi-uniform Voronoi meshes, N = 10*4**level + 2
  (2562, 40962, 163842, 655362 at levels 4, 6, 7, 8), for the BASELINE configs that the
  reference repo does not ship.  Cells are the vertices of a recursively bisected
  icosahedron, Voronoi vertices the triangle circumcentres; connectivity follows the
  MPAS grid conventions (counter-clockwise edgesOnCell, TRiSK edgesOnEdge order);
  geometry (dcEdge, dvEdge, areas, kites, angleEdge) is exact spherical geometry on the
  unit sphere.  weightsOnEdge are seeded stand-ins (throughput needs only finite values;
  parity tests use their own random values).  Entities are renumbered along a
  space-filling curve (2-D Hilbert curves on the cube faces by default, the 3-D Morton key
  on request) so that the neighbour gathers of the kernels stay local in HBM.

All connectivity is stored the way MPAS grid files store it: 1-based ids, fixed-width
arrays padded as the files pad them.  The hot path uses these raw ids as 0-based
offsets; ``to_zero_based`` gives the corrected ids of "mpas" mode.
"""
import os

import numpy as np

from .registry import REPO

FIXTURE = os.path.join(REPO, "tests", "golden", "x1.2562.mesh.npz")


class Mesh:
    def __init__(self, **arrays):
        self.__dict__.update(arrays)
        self.nCells = int(self.nEdgesOnCell.shape[0])
        self.nEdges = int(self.cellsOnEdge.shape[0])
        self.nVertices = int(self.edgesOnVertex.shape[0])

    def __repr__(self):
        return f"Mesh(nCells={self.nCells}, nEdges={self.nEdges}, nVertices={self.nVertices})"


def load_x1_2562():
    z = np.load(FIXTURE, allow_pickle=False)
    d = {k: z[k] for k in z.files}
    part = d.pop("graph_info_part_16")
    m = Mesh(**d)
    m.part = part
    m.nparts = 16
    return m


def read_graph_info_part(path, nCells):
    """mesh_loading.rg:11-22: one 0-based part id per line."""
    part = np.loadtxt(path, dtype=np.int32)
    assert part.shape == (nCells,)
    return part


# ----------------------------------------------------------------------------- geometry
def _normalize(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def _arc(a, b):
    return np.arctan2(np.linalg.norm(np.cross(a, b), axis=-1), np.sum(a * b, axis=-1))


def _tri_area(a, b, c):
    """spherical triangle area on the unit sphere (Van Oosterom & Strackee)"""
    num = np.abs(np.sum(a * np.cross(b, c), axis=-1))
    den = 1.0 + np.sum(a * b, axis=-1) + np.sum(b * c, axis=-1) + np.sum(c * a, axis=-1)
    return 2.0 * np.arctan2(num, den)


def _latlon(p):
    lat = np.arcsin(np.clip(p[..., 2], -1.0, 1.0))
    lon = np.arctan2(p[..., 1], p[..., 0])
    return lat, lon


def _morton_key(p, bits=20):
    q = ((p + 1.0) * 0.5 * ((1 << bits) - 1)).astype(np.uint64)
    key = np.zeros(p.shape[0], dtype=np.uint64)
    for b in range(bits):
        for d in range(3):
            key |= ((q[:, d] >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + d)
    return key


def _hilbert2d(x, y, order):
    """index of the integer points (x, y) in [0, 2**order)^2 along a 2-D Hilbert curve"""
    d = np.zeros(x.shape, dtype=np.int64)
    x, y = x.copy(), y.copy()
    s = 1 << (order - 1)
    while s > 0:
        rx = ((x & s) > 0).astype(np.int64)
        ry = ((y & s) > 0).astype(np.int64)
        d += s * s * ((3 * rx) ^ ry)
        m = ry == 0  # rotate the quadrant
        m1 = m & (rx == 1)
        x[m1], y[m1] = s - 1 - x[m1], s - 1 - y[m1]
        x[m], y[m] = y[m].copy(), x[m].copy()
        s >>= 1
    return d


def _cube_hilbert_key(p, order=16):
    """Sort key of unit vectors p along a 2-D Hilbert curve on each face of the circumscribed
    cube (gnomonic face coordinates), the four equatorial faces in a ring, then the poles.
    Neighbouring cells land closer together than along the 3-D Morton curve (x1.163842:
    11 % of neighbour pairs more than 64 ids apart against 14 %, 5.9 % more than 256 against
    7.2 %)."""
    a = np.abs(p)
    f = np.argmax(a, axis=1)
    sgn = np.sign(p[np.arange(len(p)), f])
    face = np.where(sgn > 0, f, f + 3)  # 0 +x, 1 +y, 2 +z, 3 -x, 4 -y, 5 -z
    u = np.empty(len(p))
    v = np.empty(len(p))
    for ax in range(3):
        m = f == ax
        o = [i for i in range(3) if i != ax]
        u[m] = p[m, o[0]] / a[m, ax]
        v[m] = p[m, o[1]] / a[m, ax]
    n = (1 << order) - 1
    xi = ((u + 1.0) * 0.5 * n).astype(np.int64)
    yi = ((v + 1.0) * 0.5 * n).astype(np.int64)
    ring = np.array([0, 1, 4, 2, 3, 5])  # face -> position: +x, +y, -x, -y, +z, -z
    return (ring[face].astype(np.int64) << (2 * order)) + _hilbert2d(xi, yi, order)


def _order_key(p, order):
    if order == "morton":
        return _morton_key(p)
    if order == "hilbert":
        return _cube_hilbert_key(p)
    raise ValueError(f"mesh order {order!r}: 'morton' or 'hilbert'")


def _icosahedron():
    t = (1.0 + 5.0 ** 0.5) / 2.0
    V = np.array([[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t], [0, 1, -t],
                  [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]], dtype=np.float64)
    F = np.array([[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2],
                  [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5],
                  [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]], dtype=np.int64)
    return _normalize(V), F


def _subdivide(V, F):
    e = np.concatenate([F[:, [0, 1]], F[:, [1, 2]], F[:, [2, 0]]])
    e.sort(axis=1)
    uniq, inv = np.unique(e, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    mid = _normalize(V[uniq[:, 0]] + V[uniq[:, 1]])
    nV = V.shape[0]
    nf = F.shape[0]
    ab, bc, ca = nV + inv[:nf], nV + inv[nf:2 * nf], nV + inv[2 * nf:]
    a, b, c = F[:, 0], F[:, 1], F[:, 2]
    F2 = np.concatenate([np.stack([a, ab, ca], 1), np.stack([b, bc, ab], 1), np.stack([c, ca, bc], 1),
                         np.stack([ab, bc, ca], 1)])
    return np.concatenate([V, mid]), F2


def icosahedral(level, seed=20211015, order=None):
    """x1.N mesh with N = 10*4**level + 2 (see module docstring).  order: the space-filling
    curve cells, vertices and edges are numbered along, "morton" (3-D Morton key of the unit
    vector) or "hilbert" (2-D Hilbert curves on the faces of the circumscribed cube); default
    env MPAS_MESH_ORDER, else "hilbert" (x1.163842: the step 0.8 % faster than with "morton",
    an 8-way split's ghost cells 3-6 % instead of 4-7 %)."""
    order = order or os.environ.get("MPAS_MESH_ORDER", "hilbert")
    V, F = _icosahedron()
    for _ in range(level):
        V, F = _subdivide(V, F)
    # renumber cells along the curve
    corder = np.argsort(_order_key(V, order), kind="stable")
    rank = np.empty_like(corder)
    rank[corder] = np.arange(corder.size)
    V = V[corder]
    F = rank[F]
    nC = V.shape[0]
    # orient triangles counter-clockwise seen from outside
    a, b, c = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    flip = np.sum(np.cross(b - a, c - a) * a, axis=1) < 0
    F[flip] = F[flip][:, [0, 2, 1]]
    # vertices (triangles) along the curve at their circumcentres
    a, b, c = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    P = _normalize(np.cross(b - a, c - a))
    vorder = np.argsort(_order_key(P, order), kind="stable")
    F, P = F[vorder], P[vorder]
    nVtx = F.shape[0]
    # edges: unique cell pairs; each has two adjacent triangles
    he = np.concatenate([F[:, [0, 1]], F[:, [1, 2]], F[:, [2, 0]]])  # half-edges (ccw in triangle)
    hv = np.concatenate([np.arange(nVtx)] * 3)
    key = np.minimum(he[:, 0], he[:, 1]) * nC + np.maximum(he[:, 0], he[:, 1])
    uk, einv = np.unique(key, return_inverse=True)
    einv = einv.reshape(-1)
    nE = uk.size
    c1 = (uk // nC).astype(np.int64)
    c2 = (uk % nC).astype(np.int64)
    mids = _normalize(V[c1] + V[c2])
    eorder = np.argsort(_order_key(mids, order), kind="stable")
    erank = np.empty_like(eorder)
    erank[eorder] = np.arange(nE)
    c1, c2, mids = c1[eorder], c2[eorder], mids[eorder]
    einv = erank[einv]
    # the two triangles of each edge: the one where the half-edge runs c1->c2 and the other
    tri_fwd = np.full(nE, -1, np.int64)
    tri_bwd = np.full(nE, -1, np.int64)
    fwd = he[:, 0] == c1[einv]
    tri_fwd[einv[fwd]] = hv[fwd]
    tri_bwd[einv[~fwd]] = hv[~fwd]
    assert (tri_fwd >= 0).all() and (tri_bwd >= 0).all()
    # MPAS: the normal points cell1 -> cell2, tangent = k x n points vertex1 -> vertex2;
    # the triangle on the right of c1->c2 (half-edge c2->c1 in ccw order) is vertex1.
    v1, v2 = tri_bwd, tri_fwd
    nvec = V[c2] - V[c1]
    tvec = P[v2] - P[v1]
    bad = np.sum(np.cross(mids, nvec) * tvec, axis=1) < 0
    v1[bad], v2[bad] = v2[bad], v1[bad].copy()
    # per-cell incident edges, counter-clockwise
    inc_e = np.concatenate([np.arange(nE), np.arange(nE)])
    inc_c = np.concatenate([c1, c2])
    o = np.lexsort((inc_e, inc_c))
    inc_e, inc_c = inc_e[o], inc_c[o]
    nEdgesOnCell = np.bincount(inc_c, minlength=nC).astype(np.int32)
    start = np.concatenate([[0], np.cumsum(nEdgesOnCell)[:-1]])
    # local angle of each incident edge midpoint around its cell
    cc = V[inc_c]
    east = _normalize(np.cross(np.array([0.0, 0.0, 1.0]), cc) + 1e-30)
    north = np.cross(cc, east)
    d = mids[inc_e] - cc
    ang = np.arctan2(np.sum(d * north, 1), np.sum(d * east, 1))
    o = np.lexsort((ang, inc_c))
    inc_e = inc_e[o]
    edgesOnCell = np.zeros((nC, 10), np.int64)
    pos = np.arange(inc_e.size) - np.repeat(start, nEdgesOnCell)
    edgesOnCell[inc_c, pos] = inc_e
    # pad like MPAS files: repeat the last valid entry
    for j in range(10):
        m = j >= nEdgesOnCell
        edgesOnCell[m, j] = edgesOnCell[m, np.maximum(nEdgesOnCell[m] - 1, 0)]
    cellsOnCell = np.where(c1[edgesOnCell] == np.arange(nC)[:, None], c2[edgesOnCell], c1[edgesOnCell])
    # verticesOnCell(i): the vertex between edgesOnCell(i) and edgesOnCell(i+1)
    nxt = edgesOnCell[np.arange(nC)[:, None], (np.arange(10)[None, :] + 1) % np.maximum(nEdgesOnCell, 1)[:, None]]
    ea, eb = edgesOnCell, nxt
    in0 = (v1[ea] == v1[eb]) | (v1[ea] == v2[eb])
    verticesOnCell = np.where(in0, v1[ea], v2[ea])
    # vertices: cells and edges of each triangle
    cellsOnVertex = F.copy()
    vt = np.concatenate([tri_fwd, tri_bwd])
    ve = np.concatenate([np.arange(nE), np.arange(nE)])
    o = np.argsort(vt, kind="stable")
    tri_e = ve[o].reshape(nVtx, 3)
    # order edgesOnVertex counter-clockwise around the vertex
    dv = mids[tri_e] - P[:, None, :]
    eastv = _normalize(np.cross(np.array([0.0, 0.0, 1.0]), P) + 1e-30)
    northv = np.cross(P, eastv)
    angv = np.arctan2(np.sum(dv * northv[:, None, :], 2), np.sum(dv * eastv[:, None, :], 2))
    tri_e = np.take_along_axis(tri_e, np.argsort(angv, axis=1), 1)
    edgesOnVertex = tri_e
    # TRiSK edgesOnEdge: edges of cell1 after e (ccw), then edges of cell2 after e
    nEdgesOnEdge = (nEdgesOnCell[c1] - 1 + nEdgesOnCell[c2] - 1).astype(np.int32)
    edgesOnEdge = np.zeros((nE, 20), np.int64)
    for side, cs in enumerate((c1, c2)):
        ne = nEdgesOnCell[cs]
        eoc = edgesOnCell[cs]
        me = np.argmax(eoc == np.arange(nE)[:, None], axis=1)
        off = np.zeros(nE, np.int64) if side == 0 else (nEdgesOnCell[c1] - 1).astype(np.int64)
        for j in range(1, 10):
            rows = np.nonzero(j < ne)[0]
            idx = (me[rows] + j) % ne[rows]
            edgesOnEdge[rows, off[rows] + j - 1] = eoc[rows, idx]
    # geometry (unit sphere)
    xCell = V
    latCell, lonCell = _latlon(V)
    latEdge, lonEdge = _latlon(mids)
    latVertex, lonVertex = _latlon(P)
    dcEdge = _arc(V[c1], V[c2])
    dvEdge = _arc(P[v1], P[v2])
    areaTriangle = _tri_area(V[F[:, 0]], V[F[:, 1]], V[F[:, 2]])
    vpos = np.arange(10)[None, :]
    vn = verticesOnCell
    vnn = verticesOnCell[np.arange(nC)[:, None], (vpos + 1) % nEdgesOnCell[:, None]]
    tri = _tri_area(np.repeat(V[:, None, :], 10, 1), P[vn], P[vnn])
    areaCell = np.sum(np.where(vpos < nEdgesOnCell[:, None], tri, 0.0), axis=1)
    # kites: vertex, midpoints of its two edges touching cell i, cell centre
    kite = np.zeros((nVtx, 3))
    for i in range(3):
        ci = cellsOnVertex[:, i]
        touch = (c1[edgesOnVertex] == ci[:, None]) | (c2[edgesOnVertex] == ci[:, None])
        two = np.argsort(~touch, axis=1, kind="stable")[:, :2]
        ea_ = np.take_along_axis(edgesOnVertex, two[:, :1], 1)[:, 0]
        eb_ = np.take_along_axis(edgesOnVertex, two[:, 1:], 1)[:, 0]
        kite[:, i] = _tri_area(P, mids[ea_], V[ci]) + _tri_area(P, V[ci], mids[eb_])
    e_east = _normalize(np.cross(np.array([0.0, 0.0, 1.0]), mids) + 1e-30)
    e_north = np.cross(mids, e_east)
    angleEdge = np.arctan2(np.sum(nvec * e_north, 1), np.sum(nvec * e_east, 1))
    rng = np.random.default_rng(seed)
    weightsOnEdge = np.where(np.arange(20)[None, :] < nEdgesOnEdge[:, None],
                             rng.uniform(-0.22, 0.22, size=(nE, 20)), 0.0)
    one = lambda a: (np.asarray(a) + 1).astype(np.int32)  # noqa: E731  (file ids are 1-based)
    eoe = np.where(np.arange(20)[None, :] < nEdgesOnEdge[:, None], edgesOnEdge + 1, 0).astype(np.int32)
    von = np.where(np.arange(10)[None, :] < nEdgesOnCell[:, None], verticesOnCell + 1, 0).astype(np.int32)
    m = Mesh(latCell=latCell, lonCell=lonCell, xCell=xCell[:, 0].copy(), yCell=xCell[:, 1].copy(),
             zCell=xCell[:, 2].copy(), meshDensity=np.ones(nC), areaCell=areaCell,
             nEdgesOnCell=nEdgesOnCell, edgesOnCell=one(edgesOnCell), cellsOnCell=one(cellsOnCell),
             verticesOnCell=von, latEdge=latEdge, lonEdge=lonEdge, xEdge=mids[:, 0].copy(),
             yEdge=mids[:, 1].copy(), zEdge=mids[:, 2].copy(), cellsOnEdge=one(np.stack([c1, c2], 1)),
             verticesOnEdge=one(np.stack([v1, v2], 1)), nEdgesOnEdge=nEdgesOnEdge, edgesOnEdge=eoe,
             weightsOnEdge=weightsOnEdge, dvEdge=dvEdge, dcEdge=dcEdge, angleEdge=angleEdge,
             latVertex=latVertex, lonVertex=lonVertex, xVertex=P[:, 0].copy(), yVertex=P[:, 1].copy(),
             zVertex=P[:, 2].copy(), areaTriangle=areaTriangle, edgesOnVertex=one(edgesOnVertex),
             cellsOnVertex=one(cellsOnVertex), kiteAreasOnVertex=kite)
    return m


def x1(ncells):
    """x1.N by its cell count"""
    level = {2562: 4, 10242: 5, 40962: 6, 163842: 7, 655362: 8}[ncells]
    return icosahedral(level)


def to_zero_based(ids, n):
    """mpas-mode connectivity: 1-based file ids -> 0-based; padding (0) -> zero slot n"""
    z = ids.astype(np.int64) - 1
    return np.where(z < 0, n, z).astype(np.int32)


# connectivity arrays of a Mesh and the entity count their ids refer to
_CONNECTIVITY = {"edgesOnCell": "nEdges", "verticesOnCell": "nVertices", "cellsOnCell": "nCells",
                 "cellsOnEdge": "nCells", "verticesOnEdge": "nVertices", "edgesOnEdge": "nEdges",
                 "edgesOnVertex": "nEdges", "cellsOnVertex": "nCells"}


def zero_based(m):
    """a copy of m with every connectivity array in mpas-mode ids (to_zero_based): the
    hot path then sees each cell among the cellsOnEdge of its own edges, which enables
    the kernels' SELF gathers (mpas_dev.h cell_pair)"""
    d = dict(m.__dict__)
    for name, count in _CONNECTIVITY.items():
        if name in d:
            d[name] = to_zero_based(d[name], getattr(m, count))
    z = Mesh(**{k: v for k, v in d.items() if k not in ("nCells", "nEdges", "nVertices")})
    return z

