"""Device-resident views at the boundary (a Regent GPU task hands over
framebuffer instances, not host arrays): mpas_upload / mpas_download given device
pointers (here torch tensors on the same GPU) move the 3-D fields device to device
(k_misc.hip k_view_copy) and stage the 2-D ones; the result equals the host-array path
bit for bit, for the reference's entity-major layout and for Legion's SOA layout
(stride_entity 8 B, stride_level 8 n B)."""
import ctypes

import numpy as np
import pytest

from helpers import compare_states, make_state
from mpasdyn import lib
from mpasdyn import mesh as M
from mpasdyn import tasks as T
from mpasdyn.registry import FIELDS

pytestmark = pytest.mark.gpu


def _dev(a, soa):
    """a torch tensor on cuda:0 holding a (SOA: levels outermost for the 3-D fields) and
    the byte strides (entity, level, component) of its view"""
    import torch
    if soa and a.ndim >= 2:
        t = torch.from_numpy(np.ascontiguousarray(np.moveaxis(a, 0, -1))).cuda()  # (..., entity)
        st = t.stride()
        e = st[-1] * a.itemsize
        rest = [s * a.itemsize for s in st[:-1]]
        return t, e, rest
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return t, None, None


@pytest.mark.parametrize("soa", [False, True])
def test_device_views_equal_host_arrays(x1_2562, soa):
    import torch
    st = make_state(M.zero_based(x1_2562), 5, "random")
    ref = st.copy()
    got = st.copy()
    with lib.Context(*st.dims()) as a, lib.Context(*st.dims()) as b:
        a.upload(st)
        keep = []
        for f in FIELDS:
            arr = st.arrays[f.name]
            se, sl, sc = st.byte_strides(f.name)
            if soa and f.kind in ("C3", "E3", "V3", "C3B"):
                t, se, rest = _dev(arr, True)
                sl = rest[0]
            elif soa and f.kind == "C3V":
                t, se, rest = _dev(arr, True)
                sl, sc = rest
            else:
                t, _, _ = _dev(arr, False)
            keep.append(t)
            torch.cuda.synchronize()
            b._check(b.lib.mpas_upload(b.h, f.index, ctypes.c_void_p(t.data_ptr()), se, sl, sc), f"upload {f.name}")
        for c in (a, b):
            T.atm_srk3(c, 720.0, 1)
            c.sync()
        a.download(ref)
        for f in FIELDS:  # download b into fresh device tensors of the same layouts
            arr = got.arrays[f.name]
            se, sl, sc = st.byte_strides(f.name)
            if soa and f.kind in ("C3", "E3", "V3", "C3B", "C3V"):
                t, se, rest = _dev(np.zeros_like(arr), True)
                sl = rest[0]
                sc = rest[1] if f.kind == "C3V" else sc
            else:
                t, _, _ = _dev(np.zeros_like(arr), False)
            torch.cuda.synchronize()
            b._check(b.lib.mpas_download(b.h, f.index, ctypes.c_void_p(t.data_ptr()), se, sl, sc),
                     f"download {f.name}")
            h = t.cpu().numpy()
            got.arrays[f.name][...] = np.moveaxis(h, -1, 0) if (soa and h.ndim >= 2 and
                                                                f.kind in ("C3", "E3", "V3", "C3B", "C3V")) else h
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]
    assert np.any(ref["tend_u"] != st["tend_u"])  # the step ran (the reference never changes u, Q7)
