"""ctypes binding of libmpasdyn.so (include/mpas_dyn.h).

The library is built in-tree (csrc/Makefile) for gfx950 only.  Loading it or creating a
context on anything but a gfx950 device fails loudly: there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

from .registry import FIELDS, BY_NAME, F_COUNT

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPAS_LIB") or os.path.join(HERE, "libmpasdyn.so")  # MPAS_LIB: A/B of two builds (tools/)

# every symbol include/mpas_dyn.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "mpas_ctx_create", "mpas_ctx_destroy", "mpas_last_error", "mpas_sync", "mpas_get_stream",
    "mpas_set_option", "mpas_get_option", "mpas_field_count", "mpas_field_id", "mpas_field_name", "mpas_field_kind",
    "mpas_field_width", "mpas_upload", "mpas_download", "mpas_fill_synthetic",
    "mpas_atm_rk_integration_setup", "mpas_atm_compute_moist_coefficients",
    "mpas_atm_compute_vert_imp_coefs", "mpas_atm_compute_dyn_tend_work",
    "mpas_atm_set_smlstep_pert_variables_work", "mpas_atm_advance_acoustic_step_work",
    "mpas_atm_divergence_damping_3d", "mpas_atm_compute_solve_diagnostics",
    "mpas_atm_rk_dynamics_substep_finish", "mpas_atm_srk3", "mpas_atm_timestep",
    "mpas_atm_recover_large_step_variables_work", "mpas_reconstruct_2d", "mpas_summarize_timestep",
    "mpas_atm_compute_output_diagnostics", "mpas_atm_advance_scalars_mono",
    "mpas_atm_compute_damping_coefs", "mpas_atm_init_coupled_diagnostics", "mpas_atm_core_init",
    "mpas_halo_ring1", "mpas_atm_compute_signs", "mpas_atm_adv_coef_compression", "mpas_atm_couple_coef_3rd_order",
    "mpas_atm_compute_mesh_scaling",
    "mpas_timing_enable", "mpas_timing_reset", "mpas_timing_count", "mpas_timing_get",
    "mpas_halo_owned", "mpas_halo_interior", "mpas_halo_plan", "mpas_set_global_ids", "mpas_rccl_unique_id", "mpas_halo_rccl",
    "mpas_halo_loopback", "mpas_halo_stats", "mpas_jw_hydrostatic", "mpas_halo_stub", "mpas_halo_socket",
]
KIND_ID = {"cell": 0, "edge": 1, "vertex": 2}

HORIZ_MIXING = {"2d_smagorinsky": 0, "2d_fixed": 1}


class MpasError(RuntimeError):
    pass


class Dims(ctypes.Structure):
    _fields_ = [("nCells", ctypes.c_int32), ("nEdges", ctypes.c_int32),
                ("nVertices", ctypes.c_int32), ("nVertLevels", ctypes.c_int32)]


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MpasError(f"{LIB_PATH} missing: build it with __graft_entry__.build() (no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
    sig = {
        "mpas_ctx_create": (i32, [ctypes.POINTER(vp), i32, ctypes.POINTER(Dims)]),
        "mpas_ctx_destroy": (i32, [vp]),
        "mpas_last_error": (ctypes.c_char_p, [vp]),
        "mpas_sync": (i32, [vp]),
        "mpas_get_stream": (i32, [vp, ctypes.POINTER(vp)]),
        "mpas_set_option": (i32, [vp, ctypes.c_char_p, i64]),
        "mpas_get_option": (i32, [vp, ctypes.c_char_p, ctypes.POINTER(i64)]),
        "mpas_field_count": (i32, []),
        "mpas_field_id": (i32, [ctypes.c_char_p]),
        "mpas_field_name": (ctypes.c_char_p, [i32]),
        "mpas_field_kind": (i32, [i32]),
        "mpas_field_width": (i32, [i32]),
        "mpas_upload": (i32, [vp, i32, vp, i64, i64, i64]),
        "mpas_download": (i32, [vp, i32, vp, i64, i64, i64]),
        "mpas_fill_synthetic": (i32, [vp, ctypes.c_uint64]),
        "mpas_atm_rk_integration_setup": (i32, [vp]),
        "mpas_atm_compute_moist_coefficients": (i32, [vp]),
        "mpas_atm_compute_vert_imp_coefs": (i32, [vp, dbl]),
        "mpas_atm_compute_dyn_tend_work": (i32, [vp, i32, dbl, i32, dbl, i32, i32]),
        "mpas_atm_set_smlstep_pert_variables_work": (i32, [vp]),
        "mpas_atm_advance_acoustic_step_work": (i32, [vp, dbl, i32]),
        "mpas_atm_divergence_damping_3d": (i32, [vp, dbl]),
        "mpas_atm_compute_solve_diagnostics": (i32, [vp, i32, i32]),
        "mpas_atm_rk_dynamics_substep_finish": (i32, [vp, i32, i32]),
        "mpas_atm_srk3": (i32, [vp, dbl, i32]),
        "mpas_atm_timestep": (i32, [vp, dbl]),
        "mpas_atm_recover_large_step_variables_work": (i32, [vp, i32, i32, dbl]),
        "mpas_reconstruct_2d": (i32, [vp, i32, i32]),
        "mpas_atm_compute_output_diagnostics": (i32, [vp]),
        "mpas_atm_advance_scalars_mono": (i32, [vp, dbl]),
        "mpas_atm_compute_damping_coefs": (i32, [vp, dbl, dbl]),
        "mpas_atm_init_coupled_diagnostics": (i32, [vp]),
        "mpas_atm_core_init": (i32, [vp]),
        "mpas_atm_compute_signs": (i32, [vp]),
        "mpas_halo_ring1": (i32, [vp, i32, i32]),
        "mpas_atm_adv_coef_compression": (i32, [vp]),
        "mpas_atm_couple_coef_3rd_order": (i32, [vp, dbl]),
        "mpas_atm_compute_mesh_scaling": (i32, [vp, i32]),
        "mpas_summarize_timestep": (i32, [vp, i32, i32, i32, ctypes.POINTER(dbl)]),
        "mpas_timing_enable": (i32, [vp, i32]),
        "mpas_timing_reset": (i32, [vp]),
        "mpas_timing_count": (i32, [vp]),
        "mpas_timing_get": (i32, [vp, i32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(i64),
                                  ctypes.POINTER(dbl)]),
        "mpas_halo_owned": (i32, [vp, i32, i32, i32]),
        "mpas_halo_interior": (i32, [vp, i32, i32, i32]),
        "mpas_halo_plan": (i32, [vp, i32, i32, vp, i32, vp, i32]),
        "mpas_set_global_ids": (i32, [vp, i32, vp, i32]),
        "mpas_rccl_unique_id": (i32, [vp]),
        "mpas_halo_rccl": (i32, [vp, i32, i32, vp]),
        "mpas_halo_loopback": (i32, [ctypes.POINTER(vp), i32]),
        "mpas_halo_stats": (i32, [vp, ctypes.POINTER(i64), ctypes.POINTER(i64)]),
        "mpas_halo_stub": (i32, [vp]),
        "mpas_halo_socket": (i32, [vp, i32, i32, ctypes.c_char_p, i32]),
        "mpas_jw_hydrostatic": (i32, [i32, i32] + [vp] * 11 + [i32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    if L.mpas_field_count() != F_COUNT:
        raise MpasError("libmpasdyn.so was built from a different mpas_fields.def")
    _lib = L
    return L


class Context:
    """One device-resident copy of the regions (cr, er, vr, vert_r) on one GPU."""

    def __init__(self, nCells, nEdges, nVertices, nVertLevels, device=0):
        self.lib = load()
        self.dims = (nCells, nEdges, nVertices, nVertLevels)
        d = Dims(nCells, nEdges, nVertices, nVertLevels)
        h = ctypes.c_void_p()
        rc = self.lib.mpas_ctx_create(ctypes.byref(h), device, ctypes.byref(d))
        if rc != 0:
            raise MpasError(f"mpas_ctx_create failed ({rc}): {self.lib.mpas_last_error(None).decode()}")
        self.h = h

    def _check(self, rc, what):
        if rc != 0:
            raise MpasError(f"{what} failed ({rc}): {self.lib.mpas_last_error(self.h).decode()}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.mpas_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---------------------------------------------------------------- residency
    def upload(self, state, names=None):
        for f in FIELDS:
            if (names is not None and f.name not in names) or f.name not in state.arrays:
                continue
            a = state.arrays[f.name]
            se, sl, sc = state.byte_strides(f.name)
            self._check(self.lib.mpas_upload(self.h, f.index, a.ctypes.data_as(ctypes.c_void_p), se, sl, sc),
                        f"upload {f.name}")

    def download(self, state, names=None):
        for f in FIELDS:
            if (names is not None and f.name not in names) or f.name not in state.arrays:
                continue
            a = state.arrays[f.name]
            se, sl, sc = state.byte_strides(f.name)
            self._check(self.lib.mpas_download(self.h, f.index, a.ctypes.data_as(ctypes.c_void_p), se, sl, sc),
                        f"download {f.name}")

    def fill_synthetic(self, seed):
        self._check(self.lib.mpas_fill_synthetic(self.h, seed), "fill_synthetic")

    def sync(self):
        self._check(self.lib.mpas_sync(self.h), "sync")

    def stream(self):
        p = ctypes.c_void_p()
        self._check(self.lib.mpas_get_stream(self.h, ctypes.byref(p)), "get_stream")
        return p.value

    def set_option(self, name, value):
        self._check(self.lib.mpas_set_option(self.h, name.encode(), int(value)), f"set_option {name}")

    def get_option(self, name):
        v = ctypes.c_int64(0)
        self._check(self.lib.mpas_get_option(self.h, name.encode(), ctypes.byref(v)), f"get_option {name}")
        return int(v.value)

    # ---------------------------------------------------------------- timing
    def timing(self, on=True):
        self._check(self.lib.mpas_timing_enable(self.h, 1 if on else 0), "timing_enable")

    def timing_reset(self):
        self._check(self.lib.mpas_timing_reset(self.h), "timing_reset")

    def timing_report(self):
        n = self.lib.mpas_timing_count(self.h)
        if n < 0:
            self._check(n, "timing_count")
        out = {}
        for i in range(n):
            name, calls, ms = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_double()
            self._check(self.lib.mpas_timing_get(self.h, i, ctypes.byref(name), ctypes.byref(calls),
                                                 ctypes.byref(ms)), "timing_get")
            out[name.value.decode()] = (calls.value, ms.value)
        return out


# ---------------------------------------------------------------------- decomposition
def setup_subdomain(ctx, dec, r):
    """give context `ctx` rank r's owned counts, global ids and halo plan of the
    mpasdyn.decomp.Decomposition `dec` (its local state is uploaded separately)"""
    L = ctx.lib
    ctx._check(L.mpas_halo_owned(ctx.h, *dec.n_owned(r)), "mpas_halo_owned")
    ctx._check(L.mpas_halo_interior(ctx.h, *dec.n_interior(r)), "mpas_halo_interior")
    ctx._check(L.mpas_halo_ring1(ctx.h, *dec.n_ring1(r)), "mpas_halo_ring1")
    # whether the ghosts close over advCellsForEdge(edgesOnCell): the tiled transport needs it
    ctx.set_option("trtile_ghosts", int(getattr(dec, "tiled_transport", False)))
    for kind, g in dec.global_ids(r).items():
        g = np.ascontiguousarray(g, dtype=np.int32)
        ctx._check(L.mpas_set_global_ids(ctx.h, KIND_ID[kind], g.ctypes.data, len(g)), "mpas_set_global_ids")
    for kind, lst in dec.plan(r).items():
        for peer, send, recv in lst:
            send = np.ascontiguousarray(send, dtype=np.int32)
            recv = np.ascontiguousarray(recv, dtype=np.int32)
            ctx._check(L.mpas_halo_plan(ctx.h, KIND_ID[kind], int(peer), send.ctypes.data, len(send),
                                        recv.ctypes.data, len(recv)), "mpas_halo_plan")


def halo_loopback(ctxs):
    """link contexts of this process (one per rank, same device) by the loopback transport"""
    L = load()
    arr = (ctypes.c_void_p * len(ctxs))(*[c.h for c in ctxs])
    rc = L.mpas_halo_loopback(arr, len(ctxs))
    if rc != 0:
        raise MpasError(f"mpas_halo_loopback failed ({rc}): {L.mpas_last_error(ctxs[0].h).decode()}")


def rccl_unique_id():
    L = load()
    buf = ctypes.create_string_buffer(128)
    rc = L.mpas_rccl_unique_id(buf)
    if rc != 0:
        raise MpasError(f"mpas_rccl_unique_id failed ({rc}): {L.mpas_last_error(None).decode()}")
    return bytes(buf.raw)


def halo_rccl(ctx, nranks, rank, uid):
    buf = ctypes.create_string_buffer(bytes(uid), 128)
    ctx._check(ctx.lib.mpas_halo_rccl(ctx.h, nranks, rank, buf), "mpas_halo_rccl")


def halo_socket(ctx, nranks, rank, host="127.0.0.1", base_port=29600):
    """the host-staged TCP transport (N processes, possibly on one GPU; mpas_dyn.h)"""
    ctx._check(ctx.lib.mpas_halo_socket(ctx.h, nranks, rank, host.encode(), base_port), "mpas_halo_socket")


def halo_stub(ctx):
    """the stub transport (measurement only: pack, a device copy for the wire, unpack)"""
    ctx._check(ctx.lib.mpas_halo_stub(ctx.h), "mpas_halo_stub")


def halo_stats(ctx):
    a, b = ctypes.c_int64(0), ctypes.c_int64(0)
    ctx._check(ctx.lib.mpas_halo_stats(ctx.h, ctypes.byref(a), ctypes.byref(b)), "mpas_halo_stats")
    return a.value, b.value

