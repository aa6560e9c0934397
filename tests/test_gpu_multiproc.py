"""The decomposed hot path in N separate PROCESSES sharing the one GPU, linked by the
library's host-staged TCP transport (mpas_halo_socket): every rank builds its own
decomposition and halo plan from the same global state, as the ranks of `bench.py --gpus
N` do, and the exchanges run the plan / pack / unpack code of the RCCL transport with the
wire replaced by host copies and sockets (RCCL itself refuses two ranks on one GPU, so the
real RCCL path runs only on the multi-GPU node).  The owned parts of the N local results,
assembled, must equal the single-context result bit for bit over whole RK3 steps --
SURVEY §8.6 "invariance check", across process boundaries.  At most 3 rank processes use
the GPU at once."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from helpers import compare_states, make_state
from mpasdyn import decomp, lib
from mpasdyn import mesh as M
from mpasdyn import tasks as T

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# one rank: rebuild the (seeded, deterministic) global state, decompose, run, save its local state
WORKER = r"""
import sys
import numpy as np
sys.path[:0] = [{repo!r} + "/mpas-regent_amd", {repo!r} + "/tests", {repo!r} + "/oracle"]
from helpers import make_state
from mpasdyn import decomp, lib
from mpasdyn import mesh as M
from mpasdyn import tasks as T
rank, n, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
L, variant, exact, overlap, steps, fdh = {L}, {variant!r}, {exact}, {overlap}, {steps}, {fdh}
m = M.load_x1_2562()
st = make_state(M.zero_based(m) if variant == "mpas0" else m, L, "random" if variant == "mpas0" else variant)
d = decomp.Decomposition(st, n)
loc = d.local_state(rank)
with lib.Context(*d.n_local(rank), st.L) as c:
    c.set_option("exact", exact)
    c.set_option("overlap", overlap)
    c.set_option("fusedamp_halo", fdh)
    lib.setup_subdomain(c, d, rank)
    c.upload(loc)
    lib.halo_socket(c, n, rank, "127.0.0.1", port)
    for s in range(steps):
        T.atm_srk3(c, 720.0, 1)
    c.sync()
    c.download(loc)
    ex, fl = lib.halo_stats(c)
np.savez(out, exchanges=ex, **{{k: loc[k] for k in loc.arrays}})
"""


def _free_port(n):
    """a base port with n free consecutive ports after it"""
    for _ in range(50):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            base = s.getsockname()[1]
        if base + n >= 65535:
            continue
        ok = True
        for p in range(base, base + n):
            with socket.socket() as t:
                try:
                    t.bind(("127.0.0.1", p))
                except OSError:
                    ok = False
                    break
        if ok:
            return base
    raise RuntimeError("no free port range")


def run_processes(st, nparts, tmp_path, L, variant, exact, overlap, steps, fdh=0):
    port = _free_port(nparts)
    code = WORKER.format(repo=REPO, L=L, variant=variant, exact=exact, overlap=overlap, steps=steps, fdh=fdh)
    outs = [str(tmp_path / f"rank{r}.npz") for r in range(nparts)]
    procs = [subprocess.Popen([sys.executable, "-c", code, str(r), str(nparts), str(port), outs[r]],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(nparts)]
    logs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=240)
            logs.append(out.decode(errors="replace")[-2000:])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)
    d = decomp.Decomposition(st, nparts)
    locs, exchanges = [], []
    for r in range(nparts):
        loc = d.local_state(r)
        with np.load(outs[r]) as z:
            for k in loc.arrays:
                loc[k] = z[k]
            exchanges.append(int(z["exchanges"]))
        locs.append(loc)
    return d.assemble(locs), exchanges


def run_single(st, exact, steps):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", exact)
        ctx.upload(st)
        for _ in range(steps):
            T.atm_srk3(ctx, 720.0, 1)
        ctx.sync()
        ctx.download(got)
    return got


@pytest.mark.parametrize("nparts,variant,L,exact,overlap,fdh", [(2, "random", 56, 1, 1, 0), (3, "mpas0", 5, 0, 1, 0),
                                                                (3, "ref", 5, 1, 0, 0), (3, "random", 56, 0, 1, 1)])
def test_srk3_processes_equal_single(x1_2562, tmp_path, nparts, variant, L, exact, overlap, fdh):
    """two RK3 steps in 2 or 3 rank processes (fdh: option fusedamp_halo)"""
    st = make_state(M.zero_based(x1_2562) if variant == "mpas0" else x1_2562, L,
                    "random" if variant == "mpas0" else variant)
    steps = 2
    ref = run_single(st, exact, steps)
    got, exchanges = run_processes(st, nparts, tmp_path, L, variant, exact, overlap, steps, fdh)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]
    assert all(e > 0 for e in exchanges) and len(set(exchanges)) == 1  # every rank ran the same exchanges


def test_socket_transport_refuses_a_second_transport(x1_2562):
    st = make_state(x1_2562, 5, "random")
    d = decomp.Decomposition(st, 2)
    with lib.Context(*d.n_local(0), st.L) as c:
        lib.setup_subdomain(c, d, 0)
        lib.halo_stub(c)
        with pytest.raises(lib.MpasError):
            lib.halo_socket(c, 2, 0, "127.0.0.1", _free_port(2))
