"""Field registry of the RK3 dynamics hot path, parsed from include/mpas_fields.def.

The same X-macro file defines the fields for the device library (csrc/mpas_dev.h), the
oracle (oracle/mpas_oracle.c) and this host package, so field ids agree everywhere.
Names are the Regent field names of data_structures.rg.
"""
import os
import re
from dataclasses import dataclass

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEF_PATH = os.path.join(REPO, "include", "mpas_fields.def")

KINDS = ["C3", "C3V", "E3", "V3", "C2F", "C2I", "E2F", "E2I", "V2F", "V2I", "C3B", "ZV"]
ENTITY = {"C3": "cell", "C3V": "cell", "C2F": "cell", "C2I": "cell", "C3B": "cell",
          "E3": "edge", "E2F": "edge", "E2I": "edge",
          "V3": "vertex", "V2F": "vertex", "V2I": "vertex", "ZV": None}


@dataclass(frozen=True)
class Field:
    index: int
    name: str
    kind: str
    width: int
    dist: str
    lo: float
    hi: float

    @property
    def entity(self):
        return ENTITY[self.kind]

    @property
    def is_3d(self):
        return self.kind in ("C3", "C3V", "E3", "V3", "C3B")

    @property
    def dtype(self):
        if self.kind in ("C2I", "E2I", "V2I"):
            return np.int32
        if self.kind == "C3B":
            return np.uint8
        return np.float64


def _parse():
    pat = re.compile(r"^MPAS_FIELD\(\s*(\w+)\s*,\s*(\w+)\s*,\s*(\d+)\s*,\s*(\w)\s*,\s*([-+0-9.eE]+)\s*,\s*([-+0-9.eE]+)\s*\)")
    out = []
    with open(DEF_PATH) as f:
        for line in f:
            m = pat.match(line.strip())
            if m:
                name, kind, w, dist, lo, hi = m.groups()
                assert kind in KINDS, kind
                out.append(Field(len(out), name, kind, int(w), dist, float(lo), float(hi)))
    return out


FIELDS = _parse()
BY_NAME = {f.name: f for f in FIELDS}
F_COUNT = len(FIELDS)
