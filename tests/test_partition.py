"""partition_regions (mesh_loading.rg:399-483) and mark_shared_cells (main.rg:48-52,
dynamics_tasks.rg:2009-2016): the vectorised host module mpasdyn/partition.py against the
literal point-set restatement oracle/partition_ref.py, the set algebra the task's comments
promise, the ring structure on a mesh whose ids mean what they say, and the two masks
main.rg's run hands the hot path (cpr = private_1[0], isShared).

Semantics (both modules): raw 1-based ids as offsets, partitionNumber
written at levels 0..L-1 only (level L is colour 0), rect2d fields written at level 0 only
and the never-written ones read as rect {(0,0),(0,0)} ("zero" policy) -- or as empty rects
("empty", the comparison policy).  Parity against Legion itself is unpinned (the reference
cannot run here); the restatements pin each other."""
import numpy as np
import pytest

import partition_ref as R
from mpasdyn import mesh as M
from mpasdyn import partition as P

L_REF = 5  # constants.rg:26


def _as_sets(A):
    return {(int(i), int(k)) for i, k in zip(*np.nonzero(A))}


@pytest.fixture(scope="module")
def ref_parts(x1_2562):
    m = x1_2562
    return P.partition_regions(m.part, m.edgesOnCell, m.cellsOnEdge, L_REF)


def test_vectorised_matches_literal_restatement(x1_2562, ref_parts):
    """every partition of every colour, point for point (x1.2562, part.16, L = 5)"""
    m = x1_2562
    lit = R.partition_regions(16, m.part.tolist(), m.edgesOnCell.tolist(), m.cellsOnEdge.tolist(), L_REF)
    for name, sets in lit.items():
        A = getattr(ref_parts, name)
        assert A.shape[0] == 16
        for c in range(16):
            assert _as_sets(A[c]) == sets[c], f"{name}[{c}]"
    assert _as_sets(P.mark_shared_cells(ref_parts)) == R.mark_shared_cells(lit)


def test_literal_restatement_empty_policy_small(x1_2562):
    """the comparison policy (unwritten rects empty) on a cut of the mesh: 4 parts, 3 levels"""
    m = M.zero_based(x1_2562)
    part = (np.arange(m.nCells) * 4 // m.nCells).astype(np.int32)
    lit = R.partition_regions(4, part.tolist(), m.edgesOnCell.tolist(), m.cellsOnEdge.tolist(), 3, "empty")
    vec = P.partition_regions(part, m.edgesOnCell, m.cellsOnEdge, 3, unwritten="empty")
    for name, sets in lit.items():
        for c in range(4):
            assert _as_sets(getattr(vec, name)[c]) == sets[c], f"{name}[{c}]"


@pytest.mark.parametrize("unwritten", ["zero", "empty"])
@pytest.mark.parametrize("ids", ["raw", "zero_based"])
def test_set_algebra(x1_2562, unwritten, ids):
    """what the task's construction guarantees whatever the ids: p is a disjoint cover of
    every point; private_1 | shared_1 = p and private_2 | shared_2 = p, each disjoint;
    shared_1 <= shared_2; ghosts lie outside p; the subsets are disjoint across colours"""
    m = x1_2562 if ids == "raw" else M.zero_based(x1_2562)
    pa = P.partition_regions(m.part, m.edgesOnCell, m.cellsOnEdge, L_REF, unwritten=unwritten)
    assert (pa.p.sum(axis=0) == 1).all()  # partition by field: every point has one colour
    for a, b in (("private_1", "shared_1"), ("private_2", "shared_2")):
        A, B = getattr(pa, a), getattr(pa, b)
        assert not (A & B).any()
        assert ((A | B) == pa.p).all()
        assert (A.sum(axis=0) <= 1).all() and (B.sum(axis=0) <= 1).all()
    assert not (pa.shared_1 & ~pa.shared_2).any()
    assert not (pa.ghost_1 & pa.p).any() and not (pa.ghost_2 & pa.p).any()
    # level L: colour 0 for every cell (partitionNumber never written there, Q6)
    assert pa.p[0, :, L_REF].all()


def test_rings_on_meaningful_ids(x1_2562):
    """with 0-based ids and empty unwritten rects the sets are the halo rings the task's
    comments describe, per column at levels 0..L-1: ghost_1 = cells across an edge of p;
    ghost_2 = cells across an edge of ghost_1 | p, minus p (rings 1 and 2); shared_1 = cells
    of p across an edge from ghost_1; shared_2 = shared_1 plus the private_1 cells across an
    edge from shared_1"""
    m = M.zero_based(x1_2562)
    pa = P.partition_regions(m.part, m.edgesOnCell, m.cellsOnEdge, L_REF, unwritten="empty")
    coe = np.asarray(m.cellsOnEdge)
    nC = m.nCells

    def across(cols):  # (nC,) bool -> cells sharing an edge with a marked cell (incl. itself)
        out = cols.copy()
        hit = cols[coe[:, 0]] | cols[coe[:, 1]]
        out[coe[hit, 0]] = True
        out[coe[hit, 1]] = True
        return out

    for c in range(16):
        p = m.part == c
        g1 = across(p) & ~p
        g2 = across(g1 | p) & ~p
        s1 = p & across(g1)
        s2 = s1 | (p & ~s1 & across(s1))
        for name, want in (("p", p), ("ghost_1", g1), ("ghost_2", g2), ("shared_1", s1), ("shared_2", s2)):
            got = getattr(pa, name)[c]
            assert (got[:, :L_REF] == want[:, None]).all(), f"{name}[{c}]"
        assert g1.sum() > 0 and s1.sum() > 0 and (s2.sum() > s1.sum())
        assert not (g1 & ~g2).any()  # ring 1 inside rings 1-2
    assert nC == 2562


def test_reference_masks(x1_2562, ref_parts):
    """the masks main.rg's run uses (x1.2562, part.16, L = 5): cpr = private_1[0] --
    every cell at level L (colour 0 by Q6), at levels 0..L-1 the part-0 cells outside
    shared_1[0], the same columns at every level; isShared = the cells marked by some
    shared_1/shared_2 at level 0.  The counts are this restatement's (regression values)."""
    m = x1_2562
    cpr, shared, pa = P.reference_masks(m.part, m.edgesOnCell, m.cellsOnEdge, L_REF)
    assert cpr.shape == (m.nCells, L_REF + 1) and cpr.dtype == np.uint8
    assert cpr[:, L_REF].all()
    cols = cpr[:, :L_REF].astype(bool)
    assert (cols == cols[:, :1]).all()
    part0 = m.part == 0
    assert not (cols[:, 0] & ~part0).any()
    assert (cols[:, 0] == (part0 & ~ref_parts.shared_1[0][:, 0])).all()
    assert shared.shape == (m.nCells,) and set(np.unique(shared)) <= {0, 1}
    marked = (ref_parts.shared_1 | ref_parts.shared_2)[:, :, 0].any(axis=0)
    assert (shared.astype(bool) == marked).all()
    assert int(cols[:, 0].sum()) == 59 and int(shared.sum()) == 2207
    assert pa.volumes(1) == {"p": 775, "e": 2541, "ghost_1_and_p": 2071, "private_1": 335, "private_2": 180,
                             "shared_1": 440, "shared_2": 595, "ghost_1": 1421, "ghost_2": 2486}


def test_apply_reference_masks(x1_2562):
    from helpers import make_state
    st = make_state(x1_2562, L_REF, "ref")
    P.apply_reference_masks(st, x1_2562)
    assert st["cprMask"][:st.nCells].sum() == 59 * L_REF + st.nCells
    assert st["isShared"][:st.nCells, 0].sum() == 2207
    assert st["cprMask"][st.nCells].sum() == 0 and st["isShared"][st.nCells, 0] == 0  # zero slot untouched
