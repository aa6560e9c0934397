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
lib.ub_gather_masked.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p]
idx, nd = cases["edge_eoe"]
for W in (64, 57, 56, 48, 32, 64, 57, 56):
    ts = []
    for rep in range(6):
        flush.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.ub_gather_masked(T.data_ptr(), idx.data_ptr(), nd, out.data_ptr(), 64, W, st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    res["edge_eoe masked W%d G64" % W] = {"ms": round(t, 4)}
lib.ub_gather_two.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
T2 = torch.rand((nE + 1) * 64, dtype=torch.float64, device=dev)
TP = torch.rand((nE + 1) * 128, dtype=torch.float64, device=dev)
for pair in (0, 1, 0, 1):
    ts = []
    for rep in range(6):
        flush.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if pair:
            lib.ub_gather_two(1, TP.data_ptr(), 0, idx.data_ptr(), nd, out.data_ptr(), 64, st)
        else:
            lib.ub_gather_two(0, T.data_ptr(), T2.data_ptr(), idx.data_ptr(), nd, out.data_ptr(), 64, st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    res["edge_eoe two fields %s G64" % ("pair16" if pair else "2x8B")] = {"ms": round(t, 4)}
lib.ub_gather_swap.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                               ctypes.c_void_p]
# correctness of the permuted layout + swap against the plain gather
perm = np.empty(64, dtype=np.int64)
perm[0::2] = np.arange(32)
perm[1::2] = np.arange(32) + 32
TPm = T.view(-1, 64)[:, torch.from_numpy(perm).to(dev)].contiguous().view(-1)  # position p holds level perm[p]
ref_out = torch.empty_like(out)
lib.ub_gather(2, T.data_ptr(), idx.data_ptr(), nd, ref_out.data_ptr(), 0, st)
lib.ub_gather_swap(TPm.data_ptr(), idx.data_ptr(), nd, out.data_ptr(), 0, st)
torch.cuda.synchronize()
got = out.view(-1, 64)[:nd][:, torch.from_numpy(np.argsort(perm)).to(dev)]
res["swap parity max|diff|"] = float((got - ref_out.view(-1, 64)[:nd]).abs().max())
for sw in (0, 1, 0, 1):
    ts = []
    for rep in range(6):
        flush.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if sw:
            lib.ub_gather_swap(TPm.data_ptr(), idx.data_ptr(), nd, out.data_ptr(), 64, st)
        else:
            lib.ub_gather(2, T.data_ptr(), idx.data_ptr(), nd, out.data_ptr(), 64, st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    res["edge_eoe 10 cols %s G64" % ("swap16" if sw else "plain8")] = {"ms": round(t, 4)}
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
lib.ub_streamp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
for mode in (0, 1, 2, 3, 4, 0, 1, 2, 3, 4):
    ts = []
    for rep in range(6):
        flush.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.ub_streamp(A.data_ptr(), B.data_ptr(), nE, D.data_ptr(), mode, st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    res["stream holes mode%d" % mode] = {"ms": round(t, 4)}
lib.ub_svar.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                        ctypes.c_void_p]
n2 = nE * 32
for mode in (0, 1, 2, 3, 4):
    for grid in (2048, 8192, n2 // 256):
        ts = []
        for rep in range(6):
            flush.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            lib.ub_svar(A.data_ptr(), B.data_ptr(), n2, D.data_ptr(), mode, grid, st)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        t = sorted(ts[1:])[len(ts[1:]) // 2]
        nb = {0: 2, 1: 3, 2: 3, 3: 2, 4: 2}[mode] * nE * 512
        res["svar mode%d grid%d" % (mode, grid)] = {"ms": round(t, 4), "TBs": round(nb / t / 1e9, 2)}
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
