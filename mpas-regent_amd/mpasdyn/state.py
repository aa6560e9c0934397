"""Host-side state in the reference's region layout.

A HostState holds one numpy array per field of the registry, indexed like the Regent
regions (data_structures.rg, regions built in main.rg:21-40):

    C3  (nCells+1, L+1)        cr[{cell, k}].f          C3V (nCells+1, L+1, W)
    E3  (nEdges+1, L+1)        er[{edge, k}].f          V3  (nVertices+1, L+1)
    C2F/C2I (nCells+1, W)      cr[{cell, 0}].f[i]       (edge/vertex likewise)
    C3B (nCells+1, L+1) uint8  explicit task masks      ZV  (L+1,)  vert_r[k].f

Row n of every entity array is the all-zero "zero slot" of the Q1 policy:
raw 1-based MPAS ids equal to n resolve to it.  It is never written.
"""
import copy

import numpy as np

from .registry import FIELDS, BY_NAME


class HostState:
    def __init__(self, nCells, nEdges, nVertices, nVertLevels, names=None):
        """names: allocate only these fields (e.g. the mesh fields of a large mesh whose
        3-D state is generated on the device); None = every field"""
        self.nCells, self.nEdges, self.nVertices = int(nCells), int(nEdges), int(nVertices)
        self.L = int(nVertLevels)
        self.arrays = {}
        for f in FIELDS:
            if names is None or f.name in names:
                self.arrays[f.name] = np.zeros(self.shape_of(f), dtype=f.dtype)

    # ------------------------------------------------------------------ layout
    def n_of(self, f):
        return {"cell": self.nCells, "edge": self.nEdges, "vertex": self.nVertices, None: 1}[f.entity]

    def shape_of(self, f):
        n = self.n_of(f) + 1
        if f.kind in ("C3", "E3", "V3", "C3B"):
            return (n, self.L + 1)
        if f.kind == "C3V":
            return (n, self.L + 1, f.width)
        if f.kind == "ZV":
            return (self.L + 1,)
        return (n, f.width)

    def __getitem__(self, name):
        return self.arrays[name]

    def __setitem__(self, name, value):
        a = self.arrays[name]
        a[...] = value

    def copy(self):
        s = copy.copy(self)
        s.arrays = {k: v.copy() for k, v in self.arrays.items()}
        return s

    def dims(self):
        return (self.nCells, self.nEdges, self.nVertices, self.L)

    def byte_strides(self, name):
        """(stride_entity, stride_level, stride_comp) in bytes, as mpas_upload takes them."""
        f = BY_NAME[name]
        a = self.arrays[name]
        if f.kind in ("C3", "E3", "V3", "C3B"):
            return a.strides[0], a.strides[1], 0
        if f.kind == "C3V":
            return a.strides[0], a.strides[1], a.strides[2]
        if f.kind == "ZV":
            return 0, a.strides[0], 0
        return a.strides[0], 0, a.strides[1]

    def check_zero_slots(self, written=()):
        """every zero slot is still zero, except those of `written` (recover_large_step
        sets the "garbage cell" of rho_zz, dynamics_tasks.rg:1790-1792)"""
        for f in FIELDS:
            if f.kind == "ZV" or f.name in written:
                continue
            a = self.arrays[f.name]
            if np.any(a[self.n_of(f)] != 0):
                raise AssertionError(f"zero slot of {f.name} was written")
