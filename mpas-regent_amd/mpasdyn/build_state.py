"""Build a HostState for a mesh: the one-time precompute that atm_core_init performs
(atm_core.rg:22-42) for the fields the hot path reads, plus synthetic 3-D state.

Variants
--------
"ref"      literal reference state: raw 1-based ids used as offsets (Q1), every field
           the reference never writes (Q2) left at 0, the derived mesh fields computed
           by restating atm_compute_signs (dynamics_tasks.rg:46-130),
           atm_adv_coef_compression (:133-269, deriv_two is a Q2 zero),
           atm_couple_coef_3rd_order (:303-325) and atm_compute_mesh_scaling (:595-646).
"physical" the same connectivity, with every Q2 field given its MPAS definition
           (invAreaCell = 1/areaCell, edgesOnCell_sign = edgesOnCellSign,
           invDcEdge = 1/dcEdge, edgesOnEdge = the grid file's edgesOnEdge, ...);
           the benchmark workload.
"random"   every fp64 input synthetic (including the Q2 and mesh-derived ones), masks and
           flags random, connectivity from the mesh: the kernel-parity workload, so every
           term of every formula is exercised with non-zero data.
3-D state comes from the counter-based generator of include/mpas_synth.h (seeded;
SURVEY §8.5 uses seed 20211015), via the oracle on the host for tests or
mpas_fill_synthetic on the device for the benchmark.
"""
import numpy as np

from .registry import BY_NAME, FIELDS
from .state import HostState

SPHERE_RADIUS = 6371229.0  # constants.rg:27
OMEGA = 7.29212E-5


def _u01(seed, fid, n, w):
    """vectorised mirror of mpas_synth.h mpas_point_hash / mpas_u01 at level 0"""
    def sm(x):
        x = (x + np.uint64(0x9E3779B97F4A7C15))
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))
    with np.errstate(over="ignore"):
        h = sm(np.uint64(seed))
        h = sm(h ^ np.uint64(fid))
        e = np.arange(n, dtype=np.uint64)[:, None]
        c = np.arange(w, dtype=np.uint64)[None, :]
        h = sm(h ^ e)
        h = sm(h ^ c)
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


# ------------------------------------------------------------- init restatements
def compute_signs(m, st):
    """atm_compute_signs, dynamics_tasks.rg:46-130 (Q1: raw ids as offsets)."""
    nC, nE, nV = m.nCells, m.nEdges, m.nVertices
    voe = np.zeros((nE + 1, 2), np.int64)
    voe[:nE] = m.verticesOnEdge
    coe = np.zeros((nE + 1, 2), np.int64)
    coe[:nE] = m.cellsOnEdge
    eov = m.edgesOnVertex.astype(np.int64)
    sgn = np.where(eov <= nE, np.where(np.arange(nV)[:, None] == voe[np.minimum(eov, nE), 1], 1.0, -1.0), 0.0)
    st["edgesOnVertexSign"][:nV] = sgn
    eoc = m.edgesOnCell.astype(np.int64)
    i = np.arange(10)[None, :]
    valid = i < m.nEdgesOnCell[:, None]
    s = np.where(eoc <= nE, np.where(np.arange(nC)[:, None] == coe[np.minimum(eoc, nE), 0], 1.0, -1.0), 0.0)
    st["edgesOnCellSign"][:nC] = np.where(valid, s, 0.0)
    # zb_cell / zb3_cell (:88-110) copy er.zb / zb3 of the initial state: left as built
    cov = np.zeros((nV + 1, 3), np.int64)
    cov[:nV] = m.cellsOnVertex
    voc = m.verticesOnCell.astype(np.int64)
    kite = np.zeros((nC, 10), np.int32)
    c = np.arange(nC)[:, None]
    vv = np.minimum(voc, nV)
    for j in (2, 1):  # first match of j = 1, 2 wins (break), so assign 2 then overwrite with 1
        kite = np.where(c == cov[vv, j], j, kite)
    kite = np.where(voc <= nV, kite, 1)
    st["kiteForCell"][:nC] = np.where(valid, kite, 0)


def adv_coef_compression_loops(m, st, dcEdge, dvEdge, deriv_two=None):
    """atm_adv_coef_compression, dynamics_tasks.rg:133-269, with its quirks:
    nAdvCellsForEdge = n is the index of the last list entry (so the last cell is never
    used), the list is capped at maxEdges-1 (:175), ids are raw (Q1), deriv_two is a Q2
    zero unless given."""
    nC, nE = m.nCells, m.nEdges
    nEoC = np.zeros(nC + 1, np.int64)
    nEoC[:nC] = m.nEdgesOnCell
    coc = np.zeros((nC + 1, 10), np.int64)
    coc[:nC] = m.cellsOnCell
    nadv = np.zeros(nE, np.int32)
    advc = np.zeros((nE, 15), np.int32)
    ac = np.zeros((nE, 15))
    ac3 = np.zeros((nE, 15))
    if deriv_two is None:
        deriv_two = np.zeros((nE, 30))
    for e in range(nE):
        cell1, cell2 = int(m.cellsOnEdge[e, 0]), int(m.cellsOnEdge[e, 1])
        if not (cell1 <= nC or cell2 <= nC):
            continue
        c1, c2 = min(cell1, nC), min(cell2, nC)
        cl = [0] * 10
        cl[0], cl[1] = cell1, cell2
        n = 1
        for i in range(nEoC[c1]):
            if coc[c1, i] != cell2:
                n += 1
                cl[n] = int(coc[c1, i])
        for ic in range(nEoC[c2]):
            add = all(cl[i] != coc[c2, ic] for i in range(n))
            if add and n < 10 - 1:
                n += 1
                cl[n] = int(coc[c2, ic])
        nadv[e] = n
        advc[e, :n] = cl[:n]
        a = np.zeros(15)
        a3 = np.zeros(15)
        j_in = 0
        for j in range(n):
            if cl[j] == cell1:
                j_in = j
        a[j_in] += deriv_two[e, 0]
        a3[j_in] += deriv_two[e, 0]
        for ic in range(nEoC[c1]):
            j_in = 0
            for j in range(n):
                if cl[j] == coc[c1, ic]:
                    j_in = j
            a[j_in] += deriv_two[e, ic * 15 + 0] if ic * 15 < 30 else 0.0
            a3[j_in] += deriv_two[e, ic * 15 + 0] if ic * 15 < 30 else 0.0
        j_in = 0
        for j in range(n):
            if cl[j] == cell2:
                j_in = j
        a[j_in] += deriv_two[e, 1]
        a3[j_in] += deriv_two[e, 1]
        for ic in range(nEoC[c2]):
            j_in = 0
            for j in range(n):
                if cl[j] == coc[c2, ic]:
                    j_in = j
            a[j_in] += deriv_two[e, ic * 15 + 1] if ic * 15 + 1 < 30 else 0.0
            a3[j_in] += deriv_two[e, ic * 15 + 1] if ic * 15 + 1 < 30 else 0.0
        for j in range(n):
            a[j] = -1.0 * (dcEdge[e] * dcEdge[e]) * a[j] / 12
            a3[j] = -1.0 * (dcEdge[e] * dcEdge[e]) * a3[j] / 12
        for target in (cell1, cell2):
            j_in = 0
            for j in range(n):
                if cl[j] == target:
                    j_in = j
            a[j_in] += 0.5
        for j in range(n):
            a[j] *= dvEdge[e]
            a3[j] *= dvEdge[e]
        ac[e], ac3[e] = a, a3
    st["nAdvCellsForEdge"][:nE, 0] = nadv
    st["advCellsForEdge"][:nE] = advc
    st["adv_coefs"][:nE] = ac
    st["adv_coefs_3rd"][:nE] = ac3 * 0.25  # atm_couple_coef_3rd_order, :313-317


def adv_coef_compression(m, st, dcEdge, dvEdge):
    """Vectorised form of adv_coef_compression_loops for deriv_two = 0 (Q2), the case
    on the path; tests/test_state.py checks it against the loop restatement."""
    nC, nE = m.nCells, m.nEdges
    nEoC = np.zeros(nC + 1, np.int64)
    nEoC[:nC] = m.nEdgesOnCell
    coc = np.zeros((nC + 1, 10), np.int64)
    coc[:nC] = m.cellsOnCell
    cell1 = m.cellsOnEdge[:, 0].astype(np.int64)
    cell2 = m.cellsOnEdge[:, 1].astype(np.int64)
    c1, c2 = np.minimum(cell1, nC), np.minimum(cell2, nC)
    cl = np.zeros((nE, 10), np.int64)
    cl[:, 0], cl[:, 1] = cell1, cell2
    n = np.ones(nE, np.int64)
    rows = np.arange(nE)
    for i in range(10):
        cand = coc[c1, i]
        add = (i < nEoC[c1]) & (cand != cell2)
        n = np.where(add, n + 1, n)
        cl[rows[add], n[add]] = cand[add]
    for ic in range(10):
        cand = coc[c2, ic]
        present = np.zeros(nE, bool)
        for i in range(10):
            present |= (i < n) & (cl[:, i] == cand)
        add = (ic < nEoC[c2]) & ~present & (n < 10 - 1)
        n = np.where(add, n + 1, n)
        cl[rows[add], n[add]] = cand[add]
    j = np.arange(15)[None, :]
    inl = j < n[:, None]
    advc = np.zeros((nE, 15), np.int32)
    advc[:, :10] = np.where(inl[:, :10], cl, 0)
    a = np.where(inl, -0.0, 0.0) * np.ones((nE, 15))  # -1.0*dc^2*0/12 for j < n
    a3 = a.copy()
    for target in (cell1, cell2):
        j_in = np.zeros(nE, np.int64)
        for jj in range(10):
            j_in = np.where((jj < n) & (cl[:, jj] == target), jj, j_in)
        a[rows, j_in] += 0.5
    a = np.where(inl, a * dvEdge[:, None], a)
    a3 = np.where(inl, a3 * dvEdge[:, None], a3)
    st["nAdvCellsForEdge"][:nE, 0] = n
    st["advCellsForEdge"][:nE] = advc
    st["adv_coefs"][:nE] = a
    st["adv_coefs_3rd"][:nE] = a3 * 0.25  # atm_couple_coef_3rd_order, :313-317


def mesh_scaling(m, st, meshDensity):
    """atm_compute_mesh_scaling with config_h_ScaleWithMesh = true (atm_core.rg:113)."""
    nC, nE = m.nCells, m.nEdges
    md = np.zeros(nC + 1)
    md[:nC] = meshDensity
    c1 = np.minimum(m.cellsOnEdge[:, 0], nC)
    c2 = np.minimum(m.cellsOnEdge[:, 1], nC)
    avg = (md[c1] + md[c2]) / 2.0
    with np.errstate(divide="ignore"):
        st["meshScalingDel2"][:nE, 0] = 1.0 / avg ** 0.25
        st["meshScalingDel4"][:nE, 0] = 1.0 / avg ** 0.75


# ------------------------------------------------------------- state builders
def connectivity(m, st):
    nC, nE, nV = m.nCells, m.nEdges, m.nVertices
    st["nEdgesOnCell"][:nC, 0] = m.nEdgesOnCell
    st["edgesOnCell"][:nC] = m.edgesOnCell
    st["verticesOnCell"][:nC] = m.verticesOnCell
    st["cellsOnEdge"][:nE] = m.cellsOnEdge
    st["verticesOnEdge"][:nE] = m.verticesOnEdge
    st["edgesOnEdge_ECP"][:nE] = m.edgesOnEdge  # mesh_loading.rg:275
    st["nEdgesOnEdge"][:nE, 0] = m.nEdgesOnEdge
    st["edgesOnVertex"][:nV] = m.edgesOnVertex
    st["cellsOnCell"][:nC] = m.cellsOnCell  # read by atm_adv_coef_compression (:133)
    st["cellsOnVertex"][:nV] = m.cellsOnVertex  # read by atm_compute_signs (:46)
    st["weightsOnEdge"][:nE] = m.weightsOnEdge
    st["kiteAreasOnVertex"][:nV] = m.kiteAreasOnVertex  # (init scales [vertexDegree] only: OOB, no effect)
    md = getattr(m, "meshDensity", None)
    st["meshDensity"][:nC, 0] = 1.0 if md is None else md  # atm_compute_damping_coefs


def geometry(m, st):
    """grid-file geometry as init_atm_case_jw leaves it (init_atm_cases.rg:87-111)"""
    nC, nE, nV = m.nCells, m.nEdges, m.nVertices
    R = SPHERE_RADIUS
    st["dvEdge"][:nE, 0] = m.dvEdge * R
    st["dcEdge"][:nE, 0] = m.dcEdge * R
    st["angleEdge"][:nE, 0] = m.angleEdge
    st["latEdge"][:nE, 0] = m.latEdge
    st["lat"][:nC, 0] = m.latCell
    st["lonEdge"][:nE, 0] = m.lonEdge
    st["lon"][:nC, 0] = m.lonCell


MESH_FIELDS = tuple(f.name for f in FIELDS if f.dist == "M" or f.kind == "ZV")


def build_state(m, nVertLevels, variant="ref", seed=20211015, oracle_fill=None, vertical=True, mesh_only=False,
                extra_names=()):
    """Return a HostState for mesh m.  ``oracle_fill(state, seed, include_mesh)`` fills the
    synthetic fields on the host (tests pass the oracle's generator); None leaves them 0
    (the benchmark fills them on the device).  mesh_only: allocate only the mesh and
    vertical-grid fields (MESH_FIELDS), for device-filled benchmark states, plus
    `extra_names` (e.g. the fields an initial state writes)."""
    names = (MESH_FIELDS + tuple(extra_names)) if mesh_only else None
    st = HostState(m.nCells, m.nEdges, m.nVertices, nVertLevels, names=names)
    nC, nE, nV, L = m.nCells, m.nEdges, m.nVertices, nVertLevels
    R = SPHERE_RADIUS
    connectivity(m, st)
    if oracle_fill is not None:
        oracle_fill(st, seed, variant == "random")
    if variant == "random":
        # integer flags and masks: random so that every branch runs
        u = _u01(seed, 1001, nC, 1)[:, 0]
        st["bdyMaskCell"][:nC, 0] = (u * 8).astype(np.int32)
        st["isShared"][:nC, 0] = (_u01(seed, 1002, nC, 1)[:, 0] < 0.3).astype(np.int32)
        st["specZoneMaskCell"][:nC, 0] = (_u01(seed, 1003, nC, 1)[:, 0] < 0.1).astype(np.float64)
        st["specZoneMaskEdge"][:nE, 0] = (_u01(seed, 1004, nE, 1)[:, 0] < 0.1).astype(np.float64)
        st["cprMask"][:nC] = (_u01(seed, 1005, nC, L + 1) < 0.8).astype(np.uint8)
        st["edgesOnEdge"][:nE] = m.edgesOnEdge
        st["kiteForCell"][:nC] = (_u01(seed, 1006, nC, 10) * 3).astype(np.int32)
        adv_coef_compression_connectivity_only(m, st)
        return st
    compute_signs(m, st)
    geometry(m, st)
    adv_coef_compression(m, st, m.dcEdge * R, m.dvEdge * R)
    mesh_scaling(m, st, m.meshDensity)
    # init_atm_cases.rg:600 with alpha_grid = 0
    st["fVertex"][:nV, 0] = 2.0 * OMEGA * np.sin(m.latVertex)
    st["cprMask"][:nC] = 1  # full-domain iteration space
    if vertical:
        rdzw, rdzu, fzm, fzp = vertical_grid(st)
        st["rdzw"], st["rdzu"], st["fzm"], st["fzp"] = rdzw, rdzu, fzm, fzp
    if variant == "physical":
        st["invAreaCell"][:nC, 0] = 1.0 / (m.areaCell * R * R)
        st["invAreaTriangle"][:nV, 0] = 1.0 / (m.areaTriangle * R * R)
        st["invDcEdge"][:nE, 0] = 1.0 / (m.dcEdge * R)
        st["invDvEdge"][:nE, 0] = 1.0 / (m.dvEdge * R)
        st["edgesOnCell_sign"][:nC] = st["edgesOnCellSign"][:nC]
        st["edgesOnVertex_sign"][:nV] = st["edgesOnVertexSign"][:nV]
        st["edgesOnEdge"][:nE] = m.edgesOnEdge
        st["kiteAreasOnVertex"][:nV] = m.kiteAreasOnVertex * R * R
        st["defc_a"][:nC] = np.where(np.arange(10)[None, :] < m.nEdgesOnCell[:, None], 0.1, 0.0)
        st["defc_b"][:nC] = np.where(np.arange(10)[None, :] < m.nEdgesOnCell[:, None], 0.05, 0.0)
    return st


def mpas_mesh_coefficients(m, st):
    """The mesh coefficients of MPAS-A's init that the reference never computes (Q2), for
    the MPAS dynamics (option physics = 2) on a 0-based mesh:

    * defc_a / defc_b (Smagorinsky deformation weights, MPAS-A init's
      atm_initialize_deformation_weights): with theta the angle of an edge normal to
      the local east of the CELL (the 3-D normal from angleEdge at the edge, seen in the
      cell's east/north frame) and s = edgesOnCell_sign,
      d_diag = u_x - v_y = sum s dv (cos 2theta u - sin 2theta v) / area,
      d_off  = u_y + v_x = sum s dv (sin 2theta u + cos 2theta v) / area
      (divergence theorem with u = u_n cos - v_t sin, v = u_n sin + v_t cos), so
      defc_a = s dv cos(2 theta) / area, defc_b = s dv sin(2 theta) / area;
    * coeffs_reconstruct (cell-centre velocity from the normal components, read by
      mpas_reconstruct_2d, dynamics_tasks.rg:1894-1948): the least-squares tangent
      vector U minimising sum_i (U . n_i - u_i)^2 over the cell's edges, in the local
      (east, north) basis, mapped to Cartesian (x, y, z) -- the role MPAS-A's RBF
      reconstruction plays (a regularised variant of the same fit)."""
    nC, nE = m.nCells, m.nEdges
    ne = np.asarray(m.nEdgesOnCell)
    eoc = np.asarray(st["edgesOnCell"][:nC], dtype=np.int64)
    on = np.arange(10)[None, :] < ne[:, None]
    e = np.where(on, eoc, 0)

    def frame(lat, lon):  # local east and north unit vectors (Cartesian)
        east = np.stack([-np.sin(lon), np.cos(lon), np.zeros_like(lon)], axis=-1)
        north = np.stack([-np.sin(lat) * np.cos(lon), -np.sin(lat) * np.sin(lon), np.cos(lat)], axis=-1)
        return east, north
    # each edge normal in 3-D from angleEdge at the edge, then its angle in the frame of
    # the cell centre (near the poles the local east rotates between edge and cell)
    ee, en = frame(np.asarray(m.latEdge), np.asarray(m.lonEdge))
    th_e = st["angleEdge"][:nE, 0]
    n3 = np.cos(th_e)[:, None] * ee + np.sin(th_e)[:, None] * en  # (nE, 3)
    lat, lon = np.asarray(m.latCell), np.asarray(m.lonCell)
    east, north = frame(lat, lon)  # (nC, 3)
    nx = np.einsum("cid,cd->ci", n3[e], east)
    ny = np.einsum("cid,cd->ci", n3[e], north)
    th = np.arctan2(ny, nx)  # (nC, 10)
    dv = st["dvEdge"][:nE, 0][e]
    sg = st["edgesOnCell_sign"][:nC]
    invA = st["invAreaCell"][:nC, 0][:, None]
    st["defc_a"][:nC] = np.where(on, sg * dv * np.cos(2.0 * th) * invA, 0.0)
    st["defc_b"][:nC] = np.where(on, sg * dv * np.sin(2.0 * th) * invA, 0.0)
    n = np.stack([np.cos(th), np.sin(th)], axis=2) * on[:, :, None]  # (nC, 10, 2)
    ntn = np.einsum("cid,cie->cde", n, n)
    coef = np.einsum("cde,cie->cdi", np.linalg.inv(ntn), n)  # (nC, 2, 10): east, north weights
    xyz = coef[:, 0, :, None] * east[:, None, :] + coef[:, 1, :, None] * north[:, None, :]  # (nC, 10, 3)
    st["coeffs_reconstruct"][:nC] = np.where(on[:, :, None], xyz, 0.0).reshape(nC, 30)


def adv_coef_compression_connectivity_only(m, st):
    """random variant: the reference's advCellsForEdge list construction, coefficients
    left to the synthetic generator"""
    nC = m.nCells
    saved_ac = st["adv_coefs"].copy()
    saved_ac3 = st["adv_coefs_3rd"].copy()
    adv_coef_compression(m, st, np.ones(m.nEdges), np.ones(m.nEdges))
    st["adv_coefs"] = saved_ac
    st["adv_coefs_3rd"] = saved_ac3


def vertical_grid(st, ztop=30000.0):
    """A smooth stretched vertical grid for the "physical" variant (init_atm_cases.rg
    derives rdzw/rdzu/fzm/fzp from zgrid the same way)."""
    L = st.L
    eta = np.linspace(0.0, 1.0, L + 1)
    zw = ztop * (0.3 * eta + 0.7 * eta ** 2)
    dzw = np.diff(zw)
    dzu = np.empty(L)
    dzu[0] = dzw[0]
    dzu[1:] = 0.5 * (dzw[1:] + dzw[:-1])
    rdzw = np.zeros(L + 1)
    rdzu = np.zeros(L + 1)
    fzm = np.zeros(L + 1)
    fzp = np.zeros(L + 1)
    rdzw[:L] = 1.0 / dzw
    rdzu[:L] = 1.0 / dzu
    fzm[1:L] = 0.5 * dzw[:-1] / dzu[1:]
    fzp[1:L] = 0.5 * dzw[1:] / dzu[1:]
    return rdzw, rdzu, fzm, fzp
