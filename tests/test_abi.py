"""The C-ABI library loads here (no GPU), exports every symbol include/mpas_dyn.h
declares, and agrees with the host registry.  No compute call is made."""
import ctypes
import os
import re

import pytest

from mpasdyn import lib
from mpasdyn.registry import FIELDS, F_COUNT

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(REPO, "include", "mpas_dyn.h")).read()
    return sorted(set(re.findall(r"\b(mpas_\w+)\s*\(", txt)))


def test_header_matches_binding_list():
    assert header_functions() == sorted(lib.EXPORTS)


def test_library_exports_every_symbol():
    L = ctypes.CDLL(lib.LIB_PATH)
    for name in header_functions():
        assert hasattr(L, name), name


def test_registry_agrees_with_library():
    L = lib.load()
    assert L.mpas_field_count() == F_COUNT
    kinds = ["C3", "C3V", "E3", "V3", "C2F", "C2I", "E2F", "E2I", "V2F", "V2I", "C3B", "ZV"]
    for f in FIELDS:
        assert L.mpas_field_id(f.name.encode()) == f.index
        assert L.mpas_field_name(f.index).decode() == f.name
        assert kinds[L.mpas_field_kind(f.index)] == f.kind
        assert L.mpas_field_width(f.index) == f.width
    assert L.mpas_field_id(b"no_such_field") < 0


def test_error_convention_without_device():
    """bad arguments are rejected with a negative code before touching a device"""
    L = lib.load()
    h = ctypes.c_void_p()
    assert L.mpas_ctx_create(ctypes.byref(h), 0, None) < 0
    bad = lib.Dims(10, 10, 10, 80)  # nVertLevels + 1 > 64
    assert L.mpas_ctx_create(ctypes.byref(h), 0, ctypes.byref(bad)) < 0
    assert L.mpas_sync(None) < 0
    assert L.mpas_atm_srk3(None, 1.0, 0) < 0


def test_library_is_gfx950_only():
    """the device code object is built for gfx950 and nothing else"""
    blob = open(lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    for other in (b"gfx942", b"gfx90a", b"gfx1100"):
        assert other not in blob


def test_bounds_build_exports_the_same_abi():
    """the bounds-checked build is a drop-in of the product library"""
    path = os.path.join(os.path.dirname(lib.LIB_PATH), "libmpasdyn_bounds.so")
    if not os.path.exists(path):
        pytest.skip("libmpasdyn_bounds.so not built (__graft_entry__.build() builds it)")
    L = ctypes.CDLL(path)
    for name in header_functions():
        assert hasattr(L, name), name
    assert b"gfx950" in open(path, "rb").read()
