"""The bounds-checked build (SURVEY §5 "bounds-checked debug kernels"; mpas_dev.h
MPAS_BOUNDS, `make -C mpas-regent_amd/csrc bounds` -> mpasdyn/libmpasdyn_bounds.so).

Every column access (colk / gather2 / gather2s / col_rd) and mesh-row load (row_ld) of every
kernel is checked against its field; an access outside it is redirected to a sink and the
C-ABI call fails with MPAS_EBOUNDS.  The library is selected with env MPAS_LIB, so each
check runs in a child process: (1) the check catches a deliberate out-of-field read;
(2) the oracle-parity tests of every task, the RK3 drivers (reference semantics, the MPAS
solver and dynamics, the transport) and the decomposed path pass under it -- no kernel
touches memory outside its fields, on meshes with raw 1-based ids (zero slot, non-SELF
gathers), 0-based ids (SELF gathers) and at LP 8, 32 and 64."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOUNDS_LIB = os.path.join(REPO, "mpas-regent_amd", "mpasdyn", "libmpasdyn_bounds.so")

PROBE = r"""
import sys
sys.path.insert(0, "mpas-regent_amd")
from mpasdyn import lib
with lib.Context(50, 150, 100, 5) as ctx:
    assert ctx.get_option("bounds") == 1, "not the bounds-checked build"
    u = ctx.get_option("bounds_units")
    print("UNITS", u >> 32, u & 0xffffffff)
    assert (u >> 32) == (u & 0xffffffff) >= 9, "a translation unit does not check"
    ctx.set_option("bounds_probe", 0)   # the zero slot itself: inside the field
    ctx.sync()
    try:
        ctx.set_option("bounds_probe", 3)
        ctx.sync()
    except lib.MpasError as e:
        print("CAUGHT", e)
    else:
        print("MISSED")
    ctx.set_option("bounds_probe", 0)   # the count was reset: the next call is clean
    ctx.sync()
    print("CLEAN")
"""


def _env():
    return dict(os.environ, MPAS_LIB=BOUNDS_LIB, PYTHONUNBUFFERED="1")


pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _bounds_lib():
    if not os.path.exists(BOUNDS_LIB):
        pytest.fail("libmpasdyn_bounds.so missing: run __graft_entry__.build() (make -C mpas-regent_amd/csrc bounds)")


def test_bounds_probe_caught():
    r = subprocess.run([sys.executable, "-c", PROBE], cwd=REPO, env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "CAUGHT" in r.stdout and "field u" in r.stdout, r.stdout + r.stderr
    assert "-6" in r.stdout or "outside their field" in r.stdout, r.stdout
    assert r.stdout.rstrip().endswith("CLEAN"), r.stdout


# the parity tests re-run under the checked build (one child pytest): every task at LP 8
# (L = 2), 64 (L = 63; raw 1-based ids: zero slot, non-SELF gathers) and 64 (L = 56, SELF
# gathers), both RK3 drivers, the MPAS solver / dynamics, the transport, the mesh tasks and
# the decomposed path (interior / boundary launches, ring-1 ghosts)
SELECTION = ["tests/test_gpu_parity.py", "tests/test_gpu_mpas_dynamics.py", "tests/test_gpu_transport.py",
             "tests/test_gpu_decomp.py"]
KSEL = ("((test_task_exact or test_task) and (random-2 or ref-63 or mpas0-56)) or "
        "(test_srk3 and not level_extremes) or test_mesh_tasks or test_atm_core_init or test_summarize or "
        "test_mpas_srk3 or test_srk3_transport or test_transport_task or test_ring1 or test_overlap_morton_mesh or "
        "test_ragged_partition or test_task_decomposed_equals_single")


def test_parity_suite_under_bounds_checks():
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-k", KSEL, *SELECTION]
    r = subprocess.run(cmd, cwd=REPO, env=_env(), capture_output=True, text=True, timeout=1100)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and "MPAS_EBOUNDS" not in r.stdout, tail
