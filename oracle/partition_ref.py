"""Literal point-set restatement of `partition_regions` (mesh_loading/mesh_loading.rg:399-483)
and `mark_shared_cells` (dynamics_tasks.rg:2009-2016, called at main.rg:48-52) --
TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product package).

Every partition is a dict colour -> Python set of (entity, level) points, and each Legion
operator is written out point by point the way its definition reads:

* partition(field, colours)[c] = { x : field(x) == c }                       (:405)
* image(R, P, f)[c]    = union over x in P[c] of the points of rect f(x) inside R (:409-454)
* preimage(R, P, f)[c] = { x in R : rect f(x) contains a point of P[c] }     (:451-469)
* |, &, - colour by colour                                                    (:419-471)

with the field values `load_mesh` leaves (mesh_loading.rg:211-247, 433-436): partitionNumber
= part[i] at levels 0..L-1 and the Q2 zero at level L; the rect2d fields written at level 0
only as {(raw id, 0), (raw id, L-1)} (Q1), and at levels 1..L the never-written value --
{(0,0),(0,0)} under the Q2 "zero" policy (one point), nothing under "empty".  This is the
independent restatement that pins the vectorised host module mpasdyn/partition.py
(tests/test_partition.py).  PARITY UNPINNED against Legion itself (not runnable here).
"""


def _rect_points(lo, hi, n, L1):
    """the points of rect {lo, hi} inside the index space {n, L1} (an int2d rect is
    inclusive at both ends; empty when lo > hi in either dimension)"""
    return {(x, y) for x in range(max(lo[0], 0), min(hi[0], n - 1) + 1)
            for y in range(max(lo[1], 0), min(hi[1], L1 - 1) + 1)}


class RectField:
    """a rect2d field of a region: written at level 0 from the raw ids, unwritten above"""

    def __init__(self, ids, L, unwritten):
        self.ids, self.L, self.unwritten = ids, L, unwritten

    def __call__(self, pt):
        i, k = pt
        if k == 0:
            r = int(self.ids[i])
            return (r, 0), (r, self.L - 1)
        if self.unwritten == "zero":
            return (0, 0), (0, 0)
        return (1, 1), (0, 0)  # empty rect


def image(n_tgt, L, P, f):
    return {c: set().union(*[_rect_points(*f(x), n_tgt, L + 1) for x in pts]) if pts else set()
            for c, pts in P.items()}


def preimage(n_src, L, P, f):
    # the rect of every source point, as its set of points (clipping changes nothing here:
    # P's points all lie inside the target index space)
    rects = [((i, k), {(x, y) for x in range(f((i, k))[0][0], f((i, k))[1][0] + 1)
                       for y in range(f((i, k))[0][1], f((i, k))[1][1] + 1)})
             for i in range(n_src) for k in range(L + 1)]
    return {c: {x for x, pts_x in rects if not pts_x.isdisjoint(pts)} for c, pts in P.items()}


def _op(a, b, fn):
    return {c: fn(a[c], b[c]) for c in a}


def partition_regions(num_partitions, part, edgesOnCell, cellsOnEdge, L, unwritten="zero"):
    nC, nE = len(part), len(cellsOnEdge)
    p = {c: set() for c in range(num_partitions)}
    for i in range(nC):
        for k in range(L + 1):
            p[int(part[i]) if k < L else 0].add((i, k))
    U = lambda a, b: a | b  # noqa: E731
    e = None
    for j in range(len(edgesOnCell[0])):
        ej = image(nE, L, p, RectField([row[j] for row in edgesOnCell], L, unwritten))
        e = ej if e is None else _op(e, ej, U)
    cellOne = RectField([row[0] for row in cellsOnEdge], L, unwritten)
    cellTwo = RectField([row[1] for row in cellsOnEdge], L, unwritten)
    ghost_1_and_p = _op(image(nC, L, e, cellOne), image(nC, L, e, cellTwo), U)
    ghost_1 = _op(ghost_1_and_p, p, lambda a, b: a - b)
    gcp_out = image(nC, L, preimage(nE, L, ghost_1_and_p, cellOne), cellTwo)
    gcp_in = image(nC, L, preimage(nE, L, ghost_1_and_p, cellTwo), cellOne)
    ghost_2 = _op(_op(gcp_in, gcp_out, U), p, lambda a, b: a - b)
    s1cp_out = image(nC, L, preimage(nE, L, ghost_1, cellOne), cellTwo)
    s1cp_in = image(nC, L, preimage(nE, L, ghost_1, cellTwo), cellOne)
    shared_1 = _op(p, _op(s1cp_out, s1cp_in, U), lambda a, b: a & b)
    private_1 = _op(p, shared_1, lambda a, b: a - b)
    s2cp_out = image(nC, L, preimage(nE, L, shared_1, cellOne), cellTwo)
    s2cp_in = image(nC, L, preimage(nE, L, shared_1, cellTwo), cellOne)
    shared_2 = _op(shared_1, _op(private_1, _op(s2cp_out, s2cp_in, U), lambda a, b: a & b), U)
    private_2 = _op(private_1, shared_2, lambda a, b: a - b)
    return {"p": p, "e": e, "ghost_1_and_p": ghost_1_and_p, "private_1": private_1, "shared_1": shared_1,
            "ghost_1": ghost_1, "private_2": private_2, "shared_2": shared_2, "ghost_2": ghost_2}


def mark_shared_cells(parts):
    """main.rg:48-52: the set of points whose isShared is true"""
    s = set()
    for c in parts["shared_1"]:
        s |= parts["shared_1"][c] | parts["shared_2"][c]
    return s
