"""mpasdyn -- MI355X-native RK3 dynamics hot path of alexaiken/mpas-regent.

The product is libmpasdyn.so (csrc/, gfx950 HIP kernels behind the C-ABI of
include/mpas_dyn.h); this package is its host side: the field registry, the
reference-layout host state, meshes and one-time precompute, the ctypes binding, and
tasks.py, which mirrors the reference's Regent task interface.
"""
from .registry import FIELDS, BY_NAME, F_COUNT  # noqa: F401
from .state import HostState  # noqa: F401
