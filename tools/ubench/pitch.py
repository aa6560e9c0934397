#!/usr/bin/env python3
"""Level-pitch microbenchmark (see pitch.hip): the column-local stream
shape and dyn_tend B's edgesOnEdge gather at the library's pitch LP = 64 and at the packed
pitch P = 58 (57 levels), on x1.163842 (nCells columns for the stream, nEdges for the gather).
Checks that both layouts give the same values, then times each kernel (median of 7, an L2 /
MALL flush between runs).

usage: python tools/ubench/pitch.py [--L 56]   (needs a GPU; pitch.so built on the CPU first:
       hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/ubench/pitch.so tools/ubench/pitch.hip)
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "..", "mpas-regent_amd")]
from mpasdyn import mesh  # noqa: E402


def lpos(P, k, NP):
    k = np.asarray(k)
    if P == 64:
        return np.where(k < 32, 2 * k, 2 * (k - 32) + 1)
    return np.where(k < NP, 2 * k, np.where(k >= 32, 2 * (k - 32) + 1, NP + k))


def pack(x, P, NP):  # x [n, L+1] -> flat [(n + 1) * P] (one slack column)
    n, nl = x.shape
    out = np.zeros((n + 1) * P)
    pos = lpos(P, np.arange(nl), NP)
    out.reshape(n + 1, P)[:n, pos] = x
    return out


def unpack(f, n, nl, P, NP):
    return f.reshape(-1, P)[:n, lpos(P, np.arange(nl), NP)]


def store_pitch(P):  # (59: the P = 58 layout read by the aligned-select kernels; 65 / 66: P = 64 with
    return 58 if P == 59 else 64 if P in (65, 66) else P  # the level-L hole / + the level-0 hole)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=56)
    a = ap.parse_args()
    nl = a.L + 1
    NP = nl - 32
    lib = ctypes.CDLL(os.path.join(HERE, "pitch.so"))
    lib.ub_stream.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_int, ctypes.c_void_p]
    lib.ub_gath.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    m = mesh.icosahedral(7)
    nC, nE = m.nCells, m.nEdges
    eoe = mesh.to_zero_based(m.edgesOnEdge, nE)[:, :10].astype(np.int32)
    eoe = np.where(eoe >= nE, nE, eoe)  # (padding ids -> the slack column)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    flush = torch.empty(768 << 20, dtype=torch.uint8, device=dev)
    rng = np.random.default_rng(1)
    res = {"L": a.L, "nCells": nC, "nEdges": nE}

    def timeit(fn):
        ts = []
        for _ in range(8):
            flush.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts[1:]))

    # gather (dyn_tend B's q: u and pv at 10 edgesOnEdge, two ids per load)
    u = rng.standard_normal((nE, nl))
    pv = rng.standard_normal((nE, nl))
    outs = {}
    for PV in (64, 58, 59, 64, 58, 59):
        P = store_pitch(PV)
        du = torch.from_numpy(pack(u, P, NP)).to(dev)
        dpv = torch.from_numpy(pack(pv, P, NP)).to(dev)
        de = torch.from_numpy(np.ascontiguousarray(eoe)).to(dev)
        do = torch.zeros(2 * (nE + 1) * P, dtype=torch.float64, device=dev)
        f = lambda: lib.ub_gath(PV, du.data_ptr(), dpv.data_ptr(), de.data_ptr(), do.data_ptr(), nE, NP, st)  # noqa
        t = timeit(f)
        o = do.cpu().numpy()
        outs[PV] = (unpack(o[:(nE + 1) * P], nE, nl, P, NP), unpack(o[(nE + 1) * P:], nE, nl, P, NP))
        res.setdefault(f"gather_P{PV}_ms", []).append(round(t, 4))
    ok_g = all(np.array_equal(outs[64][i], outs[PV][i]) for i in (0, 1) for PV in (58, 59))
    # the values themselves against numpy
    ue, pe = np.vstack([u, np.zeros((1, nl))])[eoe], np.vstack([pv, np.zeros((1, nl))])[eoe]
    s_ref = np.zeros((nE, nl))
    for i in range(10):
        s_ref = s_ref + ue[:, i] * pe[:, i]
    res["gather_values_match"] = bool(ok_g and np.allclose(outs[58][0], s_ref, rtol=1e-12, atol=1e-12))

    # stream (12 in / 2 out, and 4 in / 4 out) over cell columns
    for nin, nout, pvs in ((12, 2, (64, 58, 59, 65, 66)), (4, 4, (64, 58, 59, 65, 66)), (10, 10, (64, 65))):
        xs = [rng.standard_normal((nC, nl)) for _ in range(nin)]
        outs = {}
        for PV in pvs + pvs:
            P = store_pitch(PV)
            din = [torch.from_numpy(pack(x, P, NP)).to(dev) for x in xs]
            dout = [torch.zeros((nC + 1) * P, dtype=torch.float64, device=dev) for _ in range(nout)]
            pin = torch.tensor([t.data_ptr() for t in din], dtype=torch.int64, device=dev)
            pout = torch.tensor([t.data_ptr() for t in dout], dtype=torch.int64, device=dev)
            f = lambda: lib.ub_stream(PV, nin, pin.data_ptr(), pout.data_ptr(), nC, NP, st)  # noqa
            t = timeit(f)
            outs[PV] = [unpack(d.cpu().numpy(), nC, nl, P, NP) for d in dout]
            byts = (nin + nout) * nC * P * 8
            res.setdefault(f"stream{nin}x{nout}_P{PV}_ms", []).append(round(t, 4))
            res[f"stream{nin}x{nout}_P{PV}_TBs_of_stored_bytes"] = round(byts / t / 1e9, 2)
            res[f"stream{nin}x{nout}_P{PV}_TBs_of_57_levels"] = round((nin + nout) * nC * nl * 8 / t / 1e9, 2)
        res[f"stream{nin}x{nout}_values_match"] = all(np.array_equal(outs[64][i], outs[PV][i])
                                                      for i in range(nout) for PV in pvs if PV in (58, 59))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
