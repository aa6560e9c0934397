"""The reference's dependent partitioning and its masks: `partition_regions`
(mesh_loading/mesh_loading.rg:399-483) and `mark_shared_cells` (dynamics_tasks.rg:2009-2016)
as `main` runs them (main.rg:46-52), vectorised over colours.

What main.rg does with them: it passes `cpr = private_1[0]` to
`atm_set_smlstep_pert_variables` and `atm_divergence_damping_3d` (rk_timestep.rg:441,456;
Q6), and the isShared flags marked over `shared_1[i]` and `shared_2[i]` of all parts to the
damping's edge test (:1750).  On the device those are the fields `cprMask` (the points of
`cpr`, cell x level 0..L) and `isShared` (level 0, the point `cell1.lo` the damping reads);
`reference_masks` computes both.

Semantics restated, identical in the literal point-set oracle
`oracle/partition_ref.py`, which tests/test_partition.py checks this against:

* index spaces are int2d {n, L+1} (main.rg:21-23): points (entity, level), levels 0..L;
* `partitionNumber` is written at levels 0..L-1 only (mesh_loading.rg:221-223), so the
  level-L point of every cell is colour 0 (the Q2 zero);
* the rect2d fields `edgesOnCell0..9` (:237-246) and `cellOne` / `cellTwo` (:433-436) are
  written at level 0 only, as {(id, 0), (id, L-1)} with the RAW 1-based file id (Q1);
  an id outside [0, n) falls outside the target index space and contributes nothing
  (an image is clipped to the parent region's index space);
* the never-written rect2d values at levels 1..L follow the Q2 policy, "fresh instance
  memory reads zero": rect {(0,0), (0,0)}, which is NOT empty -- it holds the point (0,0).
  `unwritten="empty"` is the alternative policy (an empty rect), kept for comparison; the
  default "zero" is the one applied everywhere (oracle, tests, driver);
* image(R, P, f)[c] = union of f(x) over x in P[c], clipped to R;
  preimage(R, P, f)[c] = { x in R : f(x) intersects P[c] } (Legion's preimage of a range
  field: the points whose rect meets the subregion).

Sets are boolean arrays (colours, n, L+1); the reference's run is x1.2562 with 16 parts.
"""
import numpy as np


class Partitions:
    """The cell_partition_fs bundle (data_structures.rg:577-584) plus the intermediate
    partitions partition_regions prints volumes of."""

    def __init__(self, **sets):
        self.__dict__.update(sets)

    NAMES = ("private_1", "shared_1", "ghost_1", "private_2", "shared_2", "ghost_2")

    def volumes(self, colour=1):
        """the volumes partition_regions prints for colour 1 (mesh_loading.rg:407-478)"""
        v = lambda s: int(s[colour].sum())  # noqa: E731
        return {"p": v(self.p), "e": v(self.e), "ghost_1_and_p": v(self.ghost_1_and_p),
                "private_1": v(self.private_1), "private_2": v(self.private_2),
                "shared_1": v(self.shared_1), "shared_2": v(self.shared_2),
                "ghost_1": v(self.ghost_1), "ghost_2": v(self.ghost_2)}


def _rect_rows(ids, n):
    """raw ids of a level-0 rect field -> (valid, id) (ids outside [0, n) are clipped away)"""
    ids = np.asarray(ids, dtype=np.int64)
    return (ids >= 0) & (ids < n), np.where((ids >= 0) & (ids < n), ids, 0)


def _image(src, id_cols, n_tgt, L, unwritten):
    """image through rect fields written at level 0 as {(id,0),(id,L-1)} (one column of ids
    per field in id_cols, all unioned): src (C, n_src, L+1) -> (C, n_tgt, L+1)"""
    C = src.shape[0]
    out = np.zeros((C, n_tgt, L + 1), dtype=bool)
    lvl0 = src[:, :, 0]
    for ids in id_cols:
        ok, r = _rect_rows(ids, n_tgt)
        for c in range(C):
            sel = lvl0[c] & ok
            out[c, r[sel], :L] = True
    if unwritten == "zero":  # points at levels 1..L carry rect {(0,0),(0,0)}
        out[:, 0, 0] |= src[:, :, 1:].any(axis=(1, 2))
    return out


def _preimage(n_src, tgt, ids, L, unwritten):
    """preimage through one rect field written at level 0 as {(id,0),(id,L-1)}:
    tgt (C, n_tgt, L+1) -> (C, n_src, L+1)"""
    C, n_tgt = tgt.shape[0], tgt.shape[1]
    out = np.zeros((C, n_src, L + 1), dtype=bool)
    ok, r = _rect_rows(ids, n_tgt)
    col_hit = tgt[:, :, :L].any(axis=2)  # (C, n_tgt): the rect's column meets P[c]
    out[:, :, 0] = col_hit[:, r] & ok[None, :]
    if unwritten == "zero":
        out[:, :, 1:] = tgt[:, 0, 0][:, None, None]
    return out


def partition_regions(part, edgesOnCell, cellsOnEdge, nVertLevels, num_partitions=None, unwritten="zero"):
    """mesh_loading.rg:399-483.  part: (nCells,) 0-based part ids (graph.info.part.N,
    read_file :11-22); edgesOnCell (nCells, 10) and cellsOnEdge (nEdges, 2) as in the grid
    file (raw 1-based ids, Q1).  Returns Partitions with every set of the task."""
    if unwritten not in ("zero", "empty"):
        raise ValueError(f"unwritten rect policy {unwritten!r}: 'zero' or 'empty'")
    part = np.asarray(part, dtype=np.int64)
    eoc = np.asarray(edgesOnCell, dtype=np.int64)
    coe = np.asarray(cellsOnEdge, dtype=np.int64)
    nC, nE, L = len(part), len(coe), int(nVertLevels)
    C = int(num_partitions) if num_partitions is not None else int(part.max()) + 1
    # :405 p = partition(cell_region.partitionNumber, color_space)
    pn = np.zeros((nC, L + 1), dtype=np.int64)
    pn[:, :L] = part[:, None]
    p = pn[None, :, :] == np.arange(C)[:, None, None]
    # :409-419 e = union of the ten images through edgesOnCell0..9
    e = _image(p, [eoc[:, j] for j in range(eoc.shape[1])], nE, L, unwritten)
    # :442-448
    cp_one = _image(e, [coe[:, 0]], nC, L, unwritten)
    cp_two = _image(e, [coe[:, 1]], nC, L, unwritten)
    ghost_1_and_p = cp_one | cp_two
    ghost_1 = ghost_1_and_p & ~p
    # :451-455 second halo
    gep_out = _preimage(nE, ghost_1_and_p, coe[:, 0], L, unwritten)
    gep_in = _preimage(nE, ghost_1_and_p, coe[:, 1], L, unwritten)
    gcp_out = _image(gep_out, [coe[:, 1]], nC, L, unwritten)
    gcp_in = _image(gep_in, [coe[:, 0]], nC, L, unwritten)
    ghost_2 = (gcp_in | gcp_out) & ~p
    # :458-463
    s1cp_out = _image(_preimage(nE, ghost_1, coe[:, 0], L, unwritten), [coe[:, 1]], nC, L, unwritten)
    s1cp_in = _image(_preimage(nE, ghost_1, coe[:, 1], L, unwritten), [coe[:, 0]], nC, L, unwritten)
    shared_1 = p & (s1cp_out | s1cp_in)
    private_1 = p & ~shared_1
    # :466-471 (shared_2's subsets of p[c] are disjoint across colours: the dynamic_cast
    # to a disjoint partition succeeds)
    s2cp_out = _image(_preimage(nE, shared_1, coe[:, 0], L, unwritten), [coe[:, 1]], nC, L, unwritten)
    s2cp_in = _image(_preimage(nE, shared_1, coe[:, 1], L, unwritten), [coe[:, 0]], nC, L, unwritten)
    shared_2 = shared_1 | (private_1 & (s2cp_out | s2cp_in))
    if (shared_2.sum(axis=0) > 1).any():
        raise AssertionError("shared_2 not disjoint: the dynamic_cast at mesh_loading.rg:470 would fail")
    private_2 = private_1 & ~shared_2
    return Partitions(p=p, e=e, ghost_1_and_p=ghost_1_and_p, private_1=private_1, shared_1=shared_1,
                      ghost_1=ghost_1, private_2=private_2, shared_2=shared_2, ghost_2=ghost_2)


def mark_shared_cells(parts):
    """main.rg:48-52: fill(isShared, false), then mark_shared_cells(shared_1[i]) and
    (shared_2[i]) for every part (dynamics_tasks.rg:2009-2016).  Returns (nCells, L+1) bool."""
    return (parts.shared_1 | parts.shared_2).any(axis=0)


def reference_masks(part, edgesOnCell, cellsOnEdge, nVertLevels, colour=0, unwritten="zero"):
    """The masks main.rg's run hands the hot path: cprMask = private_1[colour] (main.rg:55-66
    runs colour 0 only) as (nCells, L+1) uint8, and isShared at level 0 (the point
    `cell1.lo` the damping reads, :1750) as (nCells,) int32.  Returns (cprMask, isShared,
    Partitions)."""
    parts = partition_regions(part, edgesOnCell, cellsOnEdge, nVertLevels, unwritten=unwritten)
    cpr = parts.private_1[colour].astype(np.uint8)
    shared = mark_shared_cells(parts)[:, 0].astype(np.int32)
    return cpr, shared, parts


def apply_reference_masks(st, m, colour=0, unwritten="zero"):
    """Write main.rg's masks (reference_masks over the mesh's own part file m.part) into a
    HostState: cprMask and isShared.  Returns the Partitions."""
    nC, L = st.nCells, st.L
    cpr, shared, parts = reference_masks(m.part, m.edgesOnCell, m.cellsOnEdge, L, colour, unwritten)
    st["cprMask"][:nC] = cpr
    st["isShared"][:nC, 0] = shared
    return parts
