import sys, os
sys.path[:0] = ['tests', 'mpas-regent_amd', '.']
import conftest  # noqa
from helpers import make_state
from mpasdyn import mesh as M
from mpasdyn import tasks as T
from test_gpu_decomp import run_decomposed
phys = int(sys.argv[1]) if len(sys.argv) > 1 else 0
st = make_state(M.icosahedral(4), 56, "random")
def fn(c):
    if phys:
        c.set_option("physics", phys)
    T.atm_srk3(c, 720.0, 1)
    print("---- step 2", file=sys.stderr, flush=True)
    T.atm_srk3(c, 720.0, 1)
got, stats = run_decomposed(st, 2, fn, 0)
print(stats)
