"""Option "bsplit" (fast path): dyn_tend's per-edge theta flux (and the MPAS dynamics' w flux) in
an edge kernel of their own (k_dyn_Bf) beside the edge kernel B without them.  The same
expressions on the same values, so the step is bit-identical to the unsplit fast path; and it
stays within the fast path's tolerance of the oracle."""
import numpy as np
import pytest

import oracle as O
from helpers import ZERO_SLOT_WRITTEN, compare_states, make_state
from mpasdyn import mesh as M
from mpasdyn import tasks as T
from mpasdyn import lib

pytestmark = pytest.mark.gpu


def _steps(st, bsplit, physics, n=2, transport=0):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", 0)
        ctx.set_option("physics", physics)
        ctx.set_option("transport", transport)
        assert ctx.get_option("bsplit") == 2  # (default: under the MPAS dynamics only)
        ctx.set_option("bsplit", bsplit)
        assert ctx.get_option("bsplit") == bsplit
        ctx.upload(st)
        for _ in range(n):
            T.atm_srk3(ctx, 720.0, 1)
        ctx.sync()
        ctx.download(got)
    return got


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("physics", [0, 1, 2])
def test_bsplit_bit_identical(x1_2562, L, physics):
    m = M.zero_based(x1_2562) if physics else x1_2562
    st = make_state(m, L, "random")
    a = _steps(st, 0, physics)
    b = _steps(st, 1, physics)
    bad = compare_states(b, a, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("schedule", [0, 1])
def test_bsplit_against_oracle(x1_2562, schedule):
    st = make_state(x1_2562, 56, "physical")
    ref = st.copy()
    o = O.Oracle(ref)
    o.atm_srk3(720.0, schedule)
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", 0)
        ctx.set_option("bsplit", 1)
        ctx.upload(st)
        T.atm_srk3(ctx, 720.0, schedule)
        ctx.sync()
        ctx.download(got)
    bad = compare_states(got, ref, rtol=1e-9, zero_slot_excluded=ZERO_SLOT_WRITTEN)
    assert not bad, bad[:6]
    assert np.isfinite(got["u"]).all()
