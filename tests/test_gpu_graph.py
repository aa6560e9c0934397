"""HIP-graph replay of atm_srk3 (option "graph", default on): the step is
captured once per (dt, schedule) and replayed with one hipGraphLaunch.  The replayed steps
are bit-identical to direct launches (reference semantics, the MPAS vertical solver, the
MPAS dynamics with transport), a new dt re-captures, an option change invalidates, and
per-task timing runs the launches directly."""
import numpy as np
import pytest

from helpers import compare_states, make_state
from mpasdyn import lib
from mpasdyn import mesh as M
from mpasdyn import tasks as T

pytestmark = pytest.mark.gpu


def run(st, graph, opts, dts):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("graph", graph)
        for k, v in opts.items():
            ctx.set_option(k, v)
        ctx.upload(st)
        for dt in dts:
            T.atm_srk3(ctx, dt, 1)
        ctx.sync()
        caps, launches = ctx.get_option("graph_captures"), ctx.get_option("graph_launches")
        ctx.download(got)
    return got, caps, launches


@pytest.mark.parametrize("opts", [{}, {"physics": 1}, {"physics": 2, "transport": 1}, {"exact": 1}],
                         ids=["ref", "physics1", "physics2_transport", "exact"])
def test_graph_replay_bit_identical(x1_2562, opts):
    m = M.zero_based(x1_2562) if opts.get("physics") else x1_2562
    st = make_state(m, 26, "random")
    dts = [720.0, 720.0, 720.0, 360.0, 360.0]
    ref, caps0, l0 = run(st, 0, opts, dts)
    got, caps, launches = run(st, 1, opts, dts)
    assert caps0 == 0 and l0 == 0
    assert caps == 2 and launches == len(dts)  # one capture per dt
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


def test_graph_invalidation_and_timing(x1_2562):
    st = make_state(x1_2562, 5, "random")
    with lib.Context(*st.dims()) as ctx:
        ctx.upload(st)
        T.atm_srk3(ctx, 720.0, 1)
        T.atm_srk3(ctx, 720.0, 1)
        assert ctx.get_option("graph_captures") == 1
        ctx.set_option("xcd", 32)  # any option change re-captures
        T.atm_srk3(ctx, 720.0, 1)
        assert ctx.get_option("graph_captures") == 2
        ctx.timing(True)  # per-task timing: direct launches
        T.atm_srk3(ctx, 720.0, 1)
        ctx.sync()
        assert ctx.get_option("graph_launches") == 3
        rep = ctx.timing_report()
        # (the rk_step 0 key carries the fusions' suffixes: +copy, -A)
        rk0 = [k for k in rep if k.startswith("atm_compute_dyn_tend_work[rk0")]
        assert len(rk0) == 1 and rep[rk0[0]][0] == 1
        ctx.timing(False)
        T.atm_srk3(ctx, 720.0, 1)  # the captured step is still valid
        ctx.sync()
        assert ctx.get_option("graph_captures") == 2 and ctx.get_option("graph_launches") == 4
