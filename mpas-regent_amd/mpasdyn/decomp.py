"""Horizontal domain decomposition of the RK3 hot path.

The reference splits the mesh with Legion dependent partitioning over the METIS part
file (mesh_loading.rg:399-483: owned cells by `graph.info.part`, ghost rings through
the connectivity).  Here each rank owns

* the cells of its part (a part file, mesh.read_graph_info_part, or contiguous blocks
  of the renumbered cell order),
* the edges whose cellsOnEdge(0) it owns, the vertices whose edgesOnVertex(0) it owns
  (ids resolved with the Q1 policy; an id that resolves to the zero slot falls back to
  contiguous blocks of that entity's order),

and holds as ghosts every entity its owned entities reach through an index array of
the path.  The closure is taken over exactly the index arrays the kernels follow
(ID_ARRAYS, plus cellsOnEdge(edgesOnCell), which k_prepare composes for the cell
kernels, and -- with tiled_transport -- advCellsForEdge(edgesOnCell)), so one hop from an owned entity never leaves the local set.  Every kernel
computes owned entities only; a field a kernel gathers is made fresh on the ghosts by
the device-side halo exchange right before it (csrc/mpas_halo.h; lazily, only after
some kernel wrote it).  This keeps the ref-mode ids (raw 1-based offsets, which
scramble neighbourhoods) exact: no geometric ring assumption anywhere.

Local numbering: owned entities first -- the interior ones (reaching no ghost through any
index array) before the boundary ones, each in global order -- then ghosts (global order;
for edges the ghost edges of owned cells first), then the zero slot at index n_local.
Index arrays are mapped to local ids; ids that resolve to the global zero slot, or to an
entity outside the local set (only ghost entities' own connectivity can), map to the local
zero slot.
"""
import numpy as np

from .registry import FIELDS, BY_NAME
from .state import HostState

KINDS = ("cell", "edge", "vertex")
# integer fields holding entity ids -> the entity kind they refer to
# (mirrors id_target() in csrc/mpas_ctx.cpp: these are clamped to [0, n] on upload)
ID_ARRAYS = {"edgesOnCell": "edge", "edgesOnEdge": "edge", "edgesOnEdge_ECP": "edge", "edgesOnVertex": "edge",
             "cellsOnEdge": "cell", "advCellsForEdge": "cell", "verticesOnEdge": "vertex", "verticesOnCell": "vertex",
             "cellsOnCell": "cell", "cellsOnVertex": "cell"}


# index arrays only the one-time mesh tasks of atm_core_init follow (k_mesh.hip: owned
# entities, no halo exchange beside them): part of the ghost closure, not of the
# interior / boundary split
INIT_ONLY = {"cellsOnCell", "cellsOnVertex"}


# list lengths of the variable-length index arrays: entries past them are padding the
# kernels may load (unconditionally, ahead of the accumulation) but never use
COUNTS = {"edgesOnCell": "nEdgesOnCell", "verticesOnCell": "nEdgesOnCell", "edgesOnEdge": "nEdgesOnEdge",
          "edgesOnEdge_ECP": "nEdgesOnEdge", "advCellsForEdge": "nAdvCellsForEdge", "cellsOnCell": "nEdgesOnCell"}


def active_mask(st, f, rows):
    """(len(rows), W) mask of the entries of index array f that the kernels use"""
    W = st[f].shape[1]
    if f not in COUNTS:
        return np.ones((len(rows), W), dtype=bool)
    cnt = np.asarray(st[COUNTS[f]][rows, 0], dtype=np.int64)
    return np.arange(W)[None, :] < cnt[:, None]


def _resolve(ids, n):
    """Q1 policy: any id outside [0, n] is the zero slot n"""
    ids = np.asarray(ids, dtype=np.int64)
    return np.where((ids < 0) | (ids > n), n, ids)


def _blocks(n, nparts):
    return (np.arange(n, dtype=np.int64) * nparts // max(n, 1)).astype(np.int32)


class Decomposition:
    """Partition of a global HostState into `nparts` local subdomains."""

    def __init__(self, st, nparts, cell_part=None, tiled_transport=False):
        """tiled_transport: also close the ghosts over advCellsForEdge(edgesOnCell), which
        the opt-in tiled transport (option trtile) follows -- the second cell ring across
        the boundary (x1.163842 / 8: 11 % instead of 5 % ghost cells, every exchange of a
        cell field moving that many more columns), so it is off unless asked for"""
        self.st, self.nparts = st, int(nparts)
        self.tiled_transport = bool(tiled_transport)
        self.n = {"cell": st.nCells, "edge": st.nEdges, "vertex": st.nVertices}
        nC, nE, nV = st.nCells, st.nEdges, st.nVertices
        cpart = _blocks(nC, nparts) if cell_part is None else np.asarray(cell_part, dtype=np.int32)
        assert cpart.shape == (nC,) and cpart.min() >= 0 and cpart.max() < nparts
        c0 = _resolve(st["cellsOnEdge"][:nE, 0], nC)
        epart = np.where(c0 < nC, cpart[np.minimum(c0, nC - 1)], _blocks(nE, nparts)).astype(np.int32)
        e0 = _resolve(st["edgesOnVertex"][:nV, 0], nE)
        vpart = np.where(e0 < nE, epart[np.minimum(e0, nE - 1)], _blocks(nV, nparts)).astype(np.int32)
        self.part = {"cell": cpart, "edge": epart, "vertex": vpart}
        # resolved global index arrays, (n, W)
        self.ids = {f: _resolve(st[f][:self.n[BY_NAME[f].entity]], self.n[t]) for f, t in ID_ARRAYS.items()}
        coe = np.vstack([self.ids["cellsOnEdge"], np.full((1, 2), nC)])
        eoc = self.ids["edgesOnCell"]
        self.cell_cells = np.concatenate([coe[eoc, 0], coe[eoc, 1]], axis=1)  # k_prepare's composition
        # the tiled transport's composition (k_transport.hip k_trt_*: a cell forms the
        # antidiffusive flux of each of its edges): advCellsForEdge(edgesOnCell), used entries
        self._adv = np.vstack([self.ids["advCellsForEdge"], np.full((1, self.ids["advCellsForEdge"].shape[1]), nC)])
        self._nadv = np.concatenate([np.asarray(st["nAdvCellsForEdge"][:nE, 0], dtype=np.int64), [0]])
        self._nec = np.asarray(st["nEdgesOnCell"][:nC, 0], dtype=np.int64)
        self.owned, self.local, self.g2l, self.n_int, self.n_ring1_ = [], [], [], [], []
        for r in range(self.nparts):
            own = {k: np.flatnonzero(self.part[k] == r) for k in KINDS}
            need = {k: [own[k]] for k in KINDS}
            for f, t in ID_ARRAYS.items():
                src = BY_NAME[f].entity
                need[t].append(self.ids[f][own[src]].ravel())
            need["cell"].append(self.cell_cells[own["cell"]].ravel())
            # the edges of the vertices of owned edges: solve_diagnostics' ring-1 vertices
            v1 = self.ids["verticesOnEdge"][own["edge"]].ravel()
            v1 = v1[v1 < self.n["vertex"]]
            need["edge"].append(self.ids["edgesOnVertex"][v1].ravel())
            if self.tiled_transport:
                ca, cm = self.cell_adv(own["cell"])
                need["cell"].append(ca[cm])
            # interior first: an owned entity is interior when every id its index arrays
            # (and k_prepare's composed cell ids) reach in their used entries is owned or
            # the zero slot -- its kernels use no ghost value, so they run while a halo
            # exchange is in flight (a padding entry they load and discard may be mid-update)
            isown = {}
            for k in KINDS:
                m = np.zeros(self.n[k] + 1, dtype=bool)
                m[own[k]] = True
                m[self.n[k]] = True
                isown[k] = m
            bnd = {k: np.zeros(len(own[k]), dtype=bool) for k in KINDS}
            for f, t in ID_ARRAYS.items():
                if f in INIT_ONLY:  # read by the one-time mesh tasks only, never overlapped
                    continue
                src = BY_NAME[f].entity
                use = active_mask(st, f, own[src])
                bnd[src] |= (~isown[t][self.ids[f][own[src]]] & use).any(axis=1)
            use = np.tile(active_mask(st, "edgesOnCell", own["cell"]), 2)
            bnd["cell"] |= (~isown["cell"][self.cell_cells[own["cell"]]] & use).any(axis=1)
            # (the advCellsForEdge(edgesOnCell) composition makes ghosts but not boundary
            # cells: the tiled transport moves its interior cells that reach a ghost through
            # it into its boundary launch itself, mpas_ctx.cpp trt_build)
            nint = {}
            for k in KINDS:
                nint[k] = int(np.count_nonzero(~bnd[k]))
                own[k] = np.concatenate([own[k][~bnd[k]], own[k][bnd[k]]])
            # ring-1 ghosts first among the ghosts: the edges of owned cells (used entries of
            # edgesOnCell) and the vertices of owned edges -- the launchers that also compute
            # them (mpas_halo_ring1) take one contiguous range
            first_of = {"edge": self.ids["edgesOnCell"][own["cell"]][active_mask(st, "edgesOnCell", own["cell"])],
                        "vertex": self.ids["verticesOnEdge"][own["edge"]].ravel()}
            ring1 = {}
            loc, g2l = {}, {}
            for k in KINDS:
                allk = np.unique(np.concatenate(need[k]))
                allk = allk[allk < self.n[k]]  # the zero slot is not an entity
                ghosts = np.setdiff1d(allk, own[k])
                if k in first_of:
                    first = np.isin(ghosts, first_of[k])
                    ghosts = np.concatenate([ghosts[first], ghosts[~first]])
                    ring1[k] = len(own[k]) + int(first.sum())
                loc[k] = np.concatenate([own[k], ghosts]).astype(np.int64)
                m = np.full(self.n[k] + 1, len(loc[k]), dtype=np.int64)  # default: local zero slot
                m[loc[k]] = np.arange(len(loc[k]))
                g2l[k] = m
            self.n_ring1_.append((ring1["edge"], ring1["vertex"]))
            self.owned.append(own)
            self.local.append(loc)
            self.g2l.append(g2l)
            self.n_int.append(nint)

    def cell_adv(self, cells):
        """advCellsForEdge of the edges of `cells` (len, 10 * W) and the mask of the used
        entries (edge slot below nEdgesOnCell, entry below nAdvCellsForEdge)"""
        eoc = self.ids["edgesOnCell"][cells]
        W = self._adv.shape[1]
        ids = self._adv[eoc].reshape(len(cells), -1)
        used = (np.arange(eoc.shape[1])[None, :] < self._nec[cells][:, None])[:, :, None]
        used = used & (np.arange(W)[None, None, :] < self._nadv[eoc][:, :, None])
        return ids, used.reshape(len(cells), -1)

    # ------------------------------------------------------------------ per rank
    def n_owned(self, r):
        return tuple(len(self.owned[r][k]) for k in KINDS)

    def n_ring1(self, r):
        """(owned edges + the ghost edges of owned cells, owned vertices + the ghost vertices
        of owned edges): each numbered in that order"""
        return self.n_ring1_[r]

    def n_interior(self, r):
        """owned entities of rank r whose stencils reach no ghost (numbered first)"""
        return tuple(self.n_int[r][k] for k in KINDS)

    def n_local(self, r):
        return tuple(len(self.local[r][k]) for k in KINDS)

    def local_state(self, r, st=None):
        """the rank-r HostState: every field restricted to the local entities (owned,
        then ghosts), index arrays mapped to local ids, zero slots zero"""
        st = self.st if st is None else st
        nC, nE, nV = self.n_local(r)
        names = None if len(st.arrays) == len(FIELDS) else tuple(st.arrays)
        out = HostState(nC, nE, nV, st.L, names=names)
        for f in FIELDS:
            if f.name not in st.arrays:
                continue
            a = st.arrays[f.name]
            if f.entity is None:
                out.arrays[f.name][...] = a
                continue
            gid = self.local[r][f.entity]
            b = a[gid]
            if f.name in ID_ARRAYS:
                t = ID_ARRAYS[f.name]
                b = self.g2l[r][t][_resolve(b, self.n[t])].astype(b.dtype)
            out.arrays[f.name][:len(gid)] = b
        return out

    def plan(self, r):
        """halo plan of rank r: {kind: [(peer, send_local_ids, recv_local_ids), ...]}.
        recv ids are rank r's ghosts owned by `peer`, in r's ghost order; send ids are rank
        r's owned entities that are ghosts of `peer`, in the peer's ghost order -- so the
        k-th sent column is the k-th received one on the other side."""
        out = {}
        for k in KINDS:
            own_r = self.owned[r][k]
            nown = len(own_r)
            ghosts_r = self.local[r][k][nown:]
            lst = []
            for s in range(self.nparts):
                if s == r:
                    continue
                recv_g = ghosts_r[self.part[k][ghosts_r] == s]
                ghosts_s = self.local[s][k][len(self.owned[s][k]):]
                send_g = ghosts_s[self.part[k][ghosts_s] == r]
                if len(recv_g) == 0 and len(send_g) == 0:
                    continue
                lst.append((s, self.g2l[r][k][send_g].astype(np.int32), self.g2l[r][k][recv_g].astype(np.int32)))
            out[k] = lst
        return out

    def global_ids(self, r):
        """global id of every local entity of rank r (fill_synthetic hashes these)"""
        return {k: self.local[r][k].astype(np.int32) for k in KINDS}

    def assemble(self, locals_, fields=None):
        """global HostState from the owned parts of the local states"""
        out = self.st.copy()
        for f in FIELDS:
            if fields is not None and f.name not in fields:
                continue
            if f.entity is None:
                out.arrays[f.name][...] = locals_[0].arrays[f.name]
                continue
            for r, ls in enumerate(locals_):
                own = self.owned[r][f.entity]
                b = ls.arrays[f.name][:len(own)]
                if f.name in ID_ARRAYS:
                    continue  # connectivity is not state
                out.arrays[f.name][own] = b
        return out

    def check_closure(self):
        """every id reached from an owned entity (and k_prepare's composed cell ids) is
        local to that rank; returns the number of violations (0 expected)"""
        bad = 0
        for r in range(self.nparts):
            own = self.owned[r]
            for f, t in ID_ARRAYS.items():
                tg = self.ids[f][own[BY_NAME[f].entity]].ravel()
                tg = tg[tg < self.n[t]]
                bad += int(np.sum(self.g2l[r][t][tg] >= len(self.local[r][t])))
            ca, cm = self.cell_adv(own["cell"])
            extra = (ca[cm],) if self.tiled_transport else ()
            for tg in (self.cell_cells[own["cell"]].ravel(),) + extra:
                tg = tg[tg < self.n["cell"]]
                bad += int(np.sum(self.g2l[r]["cell"][tg] >= len(self.local[r]["cell"])))
        return bad
