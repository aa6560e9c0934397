#!/usr/bin/env python3
"""Column-gather microbenchmark (see gather.hip).  Gathers the 512-B edge columns of
every cell of the x1.163842 mesh (edgesOnCell, 6 per cell) and of every edge
(edgesOnEdge, 10 per edge), with 8-B and 16-B lane loads, XCD order G in {0, 32};
also the same kernels over identity-like (streaming) indices.

usage: python tools/ubench/gather.py   (needs a GPU; builds gather.so with hipcc)
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "..", "mpas-regent_amd")]
from mpasdyn import mesh  # noqa: E402

so = os.path.join(HERE, "gather.so")
if not os.path.exists(so):  # build here (CPU) beforehand; the box only runs it
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so,
                    os.path.join(HERE, "gather.hip")], check=True)
lib = ctypes.CDLL(so)
lib.ub_gather.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                          ctypes.c_int, ctypes.c_void_p]

m = mesh.icosahedral(7)
nC, nE = m.nCells, m.nEdges
eoc = mesh.to_zero_based(m.edgesOnCell, nE)[:, :10].astype(np.int32)
eoe = mesh.to_zero_based(m.edgesOnEdge, nE)[:, :10].astype(np.int32)
dev = torch.device("cuda:0")
T = torch.rand((nE + 1) * 64, dtype=torch.float64, device=dev)
out = torch.empty(max(nC, nE) * 64, dtype=torch.float64, device=dev)
flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
cases = {
    "cell_eoc": (torch.from_numpy(np.ascontiguousarray(eoc)).to(dev), nC),
    "cell_stream": (torch.from_numpy(np.ascontiguousarray(
        (np.arange(nC)[:, None] * 3 + np.arange(10)[None, :]) % nE).astype(np.int32)).to(dev), nC),
    "edge_eoe": (torch.from_numpy(np.ascontiguousarray(eoe)).to(dev), nE),
}
st = torch.cuda.current_stream().cuda_stream
res = {}
for name, (idx, nd) in cases.items():
    for var in ((0, 1) if name != "edge_eoe" else (2, 3)):
        for G in (0, 32):
            ts = []
            for rep in range(6):
                flush.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                lib.ub_gather(var, T.data_ptr(), idx.data_ptr(), nd, out.data_ptr(), G, st)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            t = sorted(ts[1:])[len(ts[1:]) // 2]
            ng = 6 if var < 2 else 10
            req = nd * (ng + 1) * 512
            res["%s v%d G%d" % (name, var, G)] = {"ms": round(t, 4), "req_TBs": round(req / t / 1e9, 2)}
lib.ub_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
A = torch.rand(nE * 64, dtype=torch.float64, device=dev)
B = torch.rand(nE * 64, dtype=torch.float64, device=dev)
D = torch.zeros(nE * 64, dtype=torch.float64, device=dev)
for W in (56, 57, 64, 56, 57, 64):
    ts = []
    for rep in range(6):
        flush.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.ub_stream(A.data_ptr(), B.data_ptr(), nE, D.data_ptr(), W, st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    res["stream W%d" % W] = {"ms": round(t, 4), "TBs_3x456B": round(3 * nE * 456 / t / 1e9, 2)}
for fn in ("ub_stream16", "ub_stream8"):
    f = getattr(lib, fn)
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    ts = []
    for rep in range(8):
        flush.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f(A.data_ptr(), B.data_ptr(), nE, D.data_ptr(), st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    res[fn] = {"ms": round(t, 4), "TBs_rows": round(3 * nE * 512 / t / 1e9, 2)}
print(json.dumps(res, indent=1))
