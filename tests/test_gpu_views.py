"""Device-resident views at the boundary (a Regent GPU task hands over
framebuffer instances, not host arrays): mpas_upload / mpas_download given device
pointers (here hipMalloc buffers of the library's own HIP runtime: a torch tensor would do
the same, but a torch imported after the library brings a second HIP runtime into the
process) move the 3-D fields device to device
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


class DevBuf:
    """a device copy of a numpy array, through the HIP runtime libmpasdyn.so runs on"""
    _hip = None

    def __init__(self, a):
        if DevBuf._hip is None:
            lib.load()
            DevBuf._hip = ctypes.CDLL("libamdhip64.so.7")  # (the already loaded runtime)
        self.host = np.ascontiguousarray(a)
        self.p = ctypes.c_void_p()
        assert DevBuf._hip.hipMalloc(ctypes.byref(self.p), ctypes.c_size_t(max(self.host.nbytes, 8))) == 0
        assert DevBuf._hip.hipMemcpy(self.p, self.host.ctypes.data_as(ctypes.c_void_p),
                                     ctypes.c_size_t(self.host.nbytes), 1) == 0  # host to device

    def numpy(self):
        out = np.empty_like(self.host)
        assert DevBuf._hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), self.p,
                                     ctypes.c_size_t(out.nbytes), 2) == 0  # device to host
        return out

    def __del__(self):
        if self.p:
            DevBuf._hip.hipFree(self.p)


def _dev(a, soa):
    """a device buffer holding a (SOA: levels outermost for the 3-D fields) and the byte
    strides (entity, level, component) of its view"""
    if soa and a.ndim >= 2:
        t = DevBuf(np.moveaxis(a, 0, -1))  # (..., entity)
        st = t.host.strides
        return t, st[-1], list(st[:-1])
    return DevBuf(a), None, None


@pytest.mark.parametrize("soa", [False, True])
def test_device_views_equal_host_arrays(x1_2562, soa):
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
            b._check(b.lib.mpas_upload(b.h, f.index, t.p, se, sl, sc), f"upload {f.name}")
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
            b._check(b.lib.mpas_download(b.h, f.index, t.p, se, sl, sc), f"download {f.name}")
            h = t.numpy()
            got.arrays[f.name][...] = np.moveaxis(h, -1, 0) if (soa and h.ndim >= 2 and
                                                                f.kind in ("C3", "E3", "V3", "C3B", "C3V")) else h
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]
    assert np.any(ref["tend_u"] != st["tend_u"])  # the step ran (the reference never changes u, Q7)
