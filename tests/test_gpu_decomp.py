"""Decomposed hot path on one GPU: N subdomain contexts in one process, linked by the
loopback halo transport (mpas_halo_loopback; the same pack/unpack and staleness logic as
the RCCL transport), each driven by its own host thread.  The owned parts of the N
local results must equal the single-context result bit for bit -- every kernel computes
the same expression on the same (fresh) inputs -- over whole RK3 steps, per task, on
literal-ref ids, random states and mpas-mode ids.  SURVEY §8.6 "invariance check"."""
import threading

import numpy as np
import pytest

from helpers import compare_states, make_state
from mpasdyn import decomp, lib
from mpasdyn import tasks as T

pytestmark = pytest.mark.gpu

_ST = {}


def state(mesh, L, variant):
    key = (L, variant)
    if key not in _ST:
        if variant == "mpas0":
            from mpasdyn import mesh as M
            _ST[key] = make_state(M.zero_based(mesh), L, "random")
        else:
            _ST[key] = make_state(mesh, L, variant)
    return _ST[key]


def run_single(st, fn, exact):
    got = st.copy()
    with lib.Context(*st.dims()) as ctx:
        ctx.set_option("exact", exact)
        ctx.upload(st)
        fn(ctx)
        ctx.sync()
        ctx.download(got)
    return got


def run_decomposed(st, nparts, fn, exact, cell_part=None, overlap=1, tiled_transport=False):
    d = decomp.Decomposition(st, nparts, cell_part=cell_part, tiled_transport=tiled_transport)
    locs = [d.local_state(r) for r in range(nparts)]
    ctxs = [lib.Context(*d.n_local(r), st.L) for r in range(nparts)]
    try:
        for r, c in enumerate(ctxs):
            c.set_option("exact", exact)
            c.set_option("overlap", overlap)
            lib.setup_subdomain(c, d, r)
            c.upload(locs[r])
        lib.halo_loopback(ctxs)
        errs = [None] * nparts

        def drive(r):
            try:
                fn(ctxs[r])
                ctxs[r].sync()
            except Exception as e:  # noqa: BLE001 -- reported below
                errs[r] = e
        th = [threading.Thread(target=drive, args=(r,)) for r in range(nparts)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=600)
        assert all(e is None for e in errs), errs
        for r, c in enumerate(ctxs):
            c.download(locs[r])
        stats = [lib.halo_stats(c) for c in ctxs]
    finally:
        for c in ctxs:
            c.close()
    return d.assemble(locs), stats


@pytest.mark.parametrize("variant", ["ref", "random", "mpas0"])
@pytest.mark.parametrize("nparts", [2, 3])
@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("overlap", [1, 0])
def test_srk3_decomposed_equals_single(x1_2562, variant, nparts, L, overlap):
    """overlap 1: interior entities computed while the exchange runs on the halo stream"""
    st = state(x1_2562, L, variant)
    for exact in (1, 0):
        ref = run_single(st, lambda c: T.atm_srk3(c, 720.0, 1), exact)
        got, stats = run_decomposed(st, nparts, lambda c: T.atm_srk3(c, 720.0, 1), exact, overlap=overlap)
        bad = compare_states(got, ref, rtol=0.0)
        assert not bad, f"exact={exact}: {bad[:6]}"
        assert all(s[0] > 0 for s in stats)  # the halo was exercised


@pytest.mark.parametrize("cve", [1, 4, 8])
def test_dyn_tend_vertex_widths_decomposed(x1_2562, cve):
    """dyn_tend rk 0 on 3 subdomains (vertex counts not multiples of the wave's vertices:
    the last vertex wave is partial) with option cve, equal to the single context"""
    st = state(x1_2562, 56, "random")

    def fn(c):
        c.set_option("cve", cve)
        T.atm_compute_dyn_tend_work(c, 0, 720.0)
    ref = run_single(st, fn, 1)
    d = decomp.Decomposition(st, 3)
    assert cve == 1 or any(d.n_owned(r)[2] % (4 * cve) for r in range(3))
    got, _ = run_decomposed(st, 3, fn, 1)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


def test_srk3_part_file_16(x1_2562):
    """the reference's own x1.2562.graph.info.part.16 split, 16 subdomains, schedule 0"""
    st = state(x1_2562, 5, "random")
    ref = run_single(st, lambda c: T.atm_srk3(c, 720.0, 0), 1)
    got, _ = run_decomposed(st, 16, lambda c: T.atm_srk3(c, 720.0, 0), 1, cell_part=x1_2562.part)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("task", ["dyn_tend_rk0", "dyn_tend_rk1", "solve_holl", "acoustic", "div_damp", "smlstep",
                                  "recover", "reconstruct"])
def test_task_decomposed_equals_single(x1_2562, task):
    fn = {"dyn_tend_rk0": lambda c: T.atm_compute_dyn_tend_work(c, 0, 720.0),
          "dyn_tend_rk1": lambda c: T.atm_compute_dyn_tend_work(c, 1, 720.0),
          "solve_holl": lambda c: T.atm_compute_solve_diagnostics(c, True, -1),
          "acoustic": lambda c: T.atm_advance_acoustic_step_work(c, 360.0, 1),
          "div_damp": lambda c: T.atm_divergence_damping_3d(c, 240.0),
          "smlstep": lambda c: T.atm_set_smlstep_pert_variables_work(c),
          "recover": lambda c: T.atm_recover_large_step_variables_work(c, 2, 2, 240.0),
          "reconstruct": lambda c: T.mpas_reconstruct_2d(c, False, True)}[task]
    st = state(x1_2562, 56, "random")
    ref = run_single(st, fn, 1)
    for overlap in (1, 0):
        got, _ = run_decomposed(st, 3, fn, 1, overlap=overlap)
        bad = compare_states(got, ref, rtol=0.0)
        assert not bad, (overlap, bad[:6])


def test_fill_synthetic_global_ids(x1_2562):
    """decomposed synthetic fill = the global fill restricted to the local entities"""
    st = state(x1_2562, 5, "ref")
    with lib.Context(*st.dims()) as ctx:
        ctx.fill_synthetic(7)
        g = st.copy()
        ctx.download(g)
    d = decomp.Decomposition(st, 2)
    for r in range(2):
        ls = d.local_state(r)
        with lib.Context(*d.n_local(r), st.L) as ctx:
            lib.setup_subdomain(ctx, d, r)
            ctx.fill_synthetic(7)
            ctx.download(ls)
        for f in ("theta_m", "u", "pv_vertex", "zb_cell"):
            ent = {"theta_m": "cell", "u": "edge", "pv_vertex": "vertex", "zb_cell": "cell"}[f]
            gid = d.local[r][ent]
            assert np.array_equal(ls[f][:len(gid)], g[f][gid]), f


def test_rccl_transport_single_rank(x1_2562):
    """the RCCL transport end to end on the one GPU of the box: librccl resolved, a
    1-rank communicator, every exchange a (peer-less) grouped send/recv; the result
    equals the undecomposed run.  Multi-rank RCCL runs on the 8-GPU node (bench.py)."""
    st = state(x1_2562, 5, "random")
    ref = run_single(st, lambda c: T.atm_srk3(c, 720.0, 1), 1)
    d = decomp.Decomposition(st, 1)
    got = d.local_state(0)
    with lib.Context(*d.n_local(0), st.L) as ctx:
        ctx.set_option("exact", 1)
        lib.setup_subdomain(ctx, d, 0)
        ctx.upload(got)
        lib.halo_rccl(ctx, 1, 0, lib.rccl_unique_id())
        T.atm_srk3(ctx, 720.0, 1)
        ctx.sync()
        ctx.download(got)
        assert lib.halo_stats(ctx)[0] > 0
    bad = compare_states(d.assemble([got]), ref, rtol=0.0)
    assert not bad, bad[:6]


@pytest.mark.parametrize("nparts", [2, 4])
def test_overlap_morton_mesh(nparts):
    """a curve-ordered mesh (icosahedral x1.2562, the benchmark's generator): most owned
    entities are interior, so the split launches really run the interior beside the
    exchange; results stay bit-identical to the single context over two RK3 steps"""
    from mpasdyn import mesh as M
    st = make_state(M.icosahedral(4), 56, "random")
    d = decomp.Decomposition(st, nparts)
    assert all(d.n_interior(r)[0] > 0.5 * d.n_owned(r)[0] for r in range(nparts))

    def two_steps(c):
        T.atm_srk3(c, 720.0, 1)
        T.atm_srk3(c, 720.0, 1)
    ref = run_single(st, two_steps, 0)
    for overlap in (1, 0):
        got, stats = run_decomposed(st, nparts, two_steps, 0, overlap=overlap)
        bad = compare_states(got, ref, rtol=0.0)
        assert not bad, (overlap, bad[:6])


def test_ragged_partition(x1_2562):
    """very uneven subdomains (one rank owns 3 cells): ranges with few or no interior
    entities, near-empty launches; still bit-identical to the single context"""
    st = state(x1_2562, 5, "random")
    part = np.zeros(st.nCells, dtype=np.int32)
    part[-3:] = 1
    ref = run_single(st, lambda c: T.atm_srk3(c, 720.0, 1), 1)
    got, _ = run_decomposed(st, 2, lambda c: T.atm_srk3(c, 720.0, 1), 1, cell_part=part)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


def test_ring1_redundancy_saves_exchanges(x1_2562):
    """option ring1 (default 1): atm_divergence_damping_3d (reference semantics) also updates
    the ghost edges of owned cells and solve_diagnostics the ghost vertices of owned edges,
    so the acoustic step's ru_p gathers and solve's pv_vertex gathers need no exchange -- one
    exchange fewer per acoustic substep after the first and per solve_diagnostics, the same
    bits as ring1 = 0"""
    st = state(x1_2562, 56, "random")
    out = {}
    for r1 in (1, 0):
        def fn(c, r1=r1):
            c.set_option("ring1", r1)
            c.set_option("fusedamp", 0)  # (the separate damping task; fused: test_fusedamp_decomposed)
            T.atm_srk3(c, 720.0, 1)
        got, stats = run_decomposed(st, 3, fn, 0)
        out[r1] = (got, stats)
    bad = compare_states(out[1][0], out[0][0], rtol=0.0)
    assert not bad, bad[:6]
    # (the first substep's ru_p is fresh from the upload; option ntu, default on: stage 0's
    # solve_diagnostics is dead and not run, so two solves per step save their exchange)
    for s1, s0 in zip(out[1][1], out[0][1]):
        assert s0[0] - s1[0] == 6 + 2, (s0, s1)


@pytest.mark.parametrize("variant,nparts,overlap", [("random", 3, 1), ("ref", 2, 0), ("mpas0", 3, 1)])
def test_fusedamp_decomposed(x1_2562, variant, nparts, overlap):
    """options fusedamp / fusesml on a decomposed mesh (option fusedamp_halo): each damping but the
    step's last applied inside the next acoustic launch, the div exchanged where rtheta_pp
    was, ru_p fresh on the ring-1 edges without an exchange -- N subdomains equal one context
    and the separate-task decomposed run bit for bit, with fewer launches"""
    st = state(x1_2562, 56, variant)
    runs = {}
    for fd in (1, 0):
        def fn(c, fd=fd):
            c.set_option("fusedamp", fd)
            c.set_option("fusedamp_halo", 1)
            assert c.get_option("fusedamp_active") == fd
            T.atm_srk3(c, 720.0, 1)
            T.atm_srk3(c, 720.0, 0)
        runs[fd] = run_decomposed(st, nparts, fn, 0, overlap=overlap)
    ref = run_single(st, lambda c: (T.atm_srk3(c, 720.0, 1), T.atm_srk3(c, 720.0, 0)), 0)
    for fd in (1, 0):
        bad = compare_states(runs[fd][0], ref, rtol=0.0)
        assert not bad, f"fusedamp={fd}: {bad[:6]}"
    for s1, s0 in zip(runs[1][1], runs[0][1]):  # the same number of exchanges (div for rtheta_pp)
        assert s1[0] == s0[0], (s1, s0)


def test_ring1_rank_without_boundary_edges(x1_2562):
    """a rank that owns no edge (one cell none of whose edges has it as cellsOnEdge(0);
    mpas-mode ids): its interior edge range equals its owned one (both empty) while it has
    ring-1 ghost edges.  Only the launch after the exchange may extend the damping over the
    ring-1 edges -- extending the interior launch too applied the increment twice"""
    st = state(x1_2562, 5, "mpas0")
    coe = st["cellsOnEdge"][:st.nEdges]
    owners = np.zeros(st.nCells, dtype=np.int64)
    np.add.at(owners, coe[:, 0], 1)
    lone = int(np.nonzero(owners == 0)[0][0])
    part = np.zeros(st.nCells, dtype=np.int32)
    part[lone] = 1
    d = decomp.Decomposition(st, 2, cell_part=part)
    assert d.n_owned(1)[1] == 0 and d.n_interior(1)[1] == 0 and d.n_ring1(1)[0] > 0
    ref = run_single(st, lambda c: T.atm_srk3(c, 720.0, 1), 1)
    got, _ = run_decomposed(st, 2, lambda c: T.atm_srk3(c, 720.0, 1), 1, cell_part=part, overlap=1)
    bad = compare_states(got, ref, rtol=0.0)
    assert not bad, bad[:6]


def test_stub_transport_graph_replay(x1_2562):
    """a decomposed context on the stub transport (tools/rank_sim.py: one rank's launch
    sequence on one GPU) with option graph_halo: the step is captured once the halo
    bookkeeping at its start repeats, and the replays leave the same bits and the same
    exchange counts as eager steps (the ghosts hold stub values, identical in both runs)"""
    st = state(x1_2562, 56, "random")
    d = decomp.Decomposition(st, 4)
    out = {}
    for graph in (1, 0):
        loc = d.local_state(1)
        with lib.Context(*d.n_local(1), st.L) as ctx:
            lib.setup_subdomain(ctx, d, 1)
            lib.halo_stub(ctx)
            assert ctx.get_option("graph_halo") == 2  # (the default: on for the stub)
            ctx.set_option("graph_halo", 2 if graph else 0)
            ctx.upload(loc)
            for _ in range(8):
                T.atm_srk3(ctx, 720.0, 1)
            ctx.sync()
            ctx.download(loc)
            out[graph] = (loc, lib.halo_stats(ctx), ctx.get_option("graph_captures"), ctx.get_option("graph_launches"))
    bad = compare_states(out[1][0], out[0][0], rtol=0.0)
    assert not bad, bad[:6]
    assert out[1][1] == out[0][1]
    assert out[1][2] == 1 and out[1][3] >= 3 and out[0][2] == 0


@pytest.mark.parametrize("between", ["solve", "upload", "fusedamp_halo", "schedules"])
def test_stub_graph_start_states(x1_2562, between):
    """graph_halo keys a captured step on the halo state at the step's start: a
    standalone task between steps (solve_diagnostics: it writes fields the step exchanges), an
    upload between steps, fusedamp_halo with the graph, and alternating schedules (two keys) each give start states other than the
    steady one; replays leave the same bits and exchange counts as eager steps"""
    st = state(x1_2562, 56, "random")
    d = decomp.Decomposition(st, 4)
    out = {}
    for graph in (1, 0):
        loc = d.local_state(1)
        with lib.Context(*d.n_local(1), st.L) as ctx:
            lib.setup_subdomain(ctx, d, 1)
            lib.halo_stub(ctx)
            ctx.set_option("graph_halo", graph)
            if between == "fusedamp_halo":  # (the default is 1: the non-fused decomposed path under replay)
                ctx.set_option("fusedamp_halo", 0)
            ctx.upload(loc)
            for i in range(9):
                T.atm_srk3(ctx, 720.0, 1 if between != "schedules" or i % 2 else 0)
                if between == "solve" and i % 3 != 2:  # (two start states alternate with the steady one)
                    T.atm_compute_solve_diagnostics(ctx, False, 2)
                if between == "upload" and i == 4:
                    ctx.upload(loc, names=["u", "theta_m"])
            ctx.sync()
            ctx.download(loc)
            out[graph] = (loc, lib.halo_stats(ctx), ctx.get_option("graph_captures"), ctx.get_option("graph_launches"))
    bad = compare_states(out[1][0], out[0][0], rtol=0.0)
    assert not bad, bad[:6]
    assert out[1][1] == out[0][1]
    assert out[1][2] >= 1 and out[1][3] >= 2 and out[0][2] == 0


@pytest.mark.parametrize("overlap", [0, 1])
def test_stub_capture_refused_falls_back(x1_2562, overlap):
    """a transport that refuses the capture of a decomposed step (test hook
    stub_refuse_capture): the capture is abandoned -- with the overlap on, after the halo
    stream was forked, which must be joined back so that the capture can be ended
    -- the step runs again eagerly, graph_fallbacks counts it once, the user's graph_halo is
    kept, no race is left behind, and every step equals the eager run bit for bit"""
    st = state(x1_2562, 56, "random")
    d = decomp.Decomposition(st, 4)
    out = {}
    for refuse in (1, 0):
        loc = d.local_state(1)
        with lib.Context(*d.n_local(1), st.L) as ctx:
            lib.setup_subdomain(ctx, d, 1)
            lib.halo_stub(ctx)
            ctx.set_option("overlap", overlap)
            ctx.set_option("graph_halo", 2 if refuse else 0)
            ctx.set_option("stub_refuse_capture", refuse)
            ctx.upload(loc)
            for _ in range(5):
                T.atm_srk3(ctx, 720.0, 1)
            T.atm_compute_solve_diagnostics(ctx, False, 2)  # (a task after the fallback: no stale race)
            ctx.sync()
            ctx.download(loc)
            out[refuse] = (loc, lib.halo_stats(ctx), ctx.get_option("graph_fallbacks"),
                           ctx.get_option("graph_captures"), ctx.get_option("graph_halo"),
                           ctx.get_option("graph_refused"))
    bad = compare_states(out[1][0], out[0][0], rtol=0.0)
    assert not bad, bad[:6]
    assert out[1][1] == out[0][1]
    assert out[1][2] == 1 and out[1][3] == 0, out[1][2:]
    assert out[1][4] == 2 and out[1][5] == 1  # (the option as set; the refusal recorded apart)
    assert out[0][2] == 0


def test_rccl_graph_capture_single_rank(x1_2562):
    """graph_halo = 1 (opt-in for RCCL; the default 2 leaves RCCL steps eager) with the RCCL
    transport: a 1-rank communicator's grouped send / recv captured into the step's graph and
    replayed; bit-identical to eager steps, no fallback to eager (graph_fallbacks), the same
    exchange counts; under the default no step is captured"""
    st = state(x1_2562, 56, "random")
    d = decomp.Decomposition(st, 1)
    out = {}
    for graph in (1, 0):
        got = d.local_state(0)
        with lib.Context(*d.n_local(0), st.L) as ctx:
            lib.setup_subdomain(ctx, d, 0)
            ctx.upload(got)
            lib.halo_rccl(ctx, 1, 0, lib.rccl_unique_id())
            assert ctx.get_option("graph_halo") == 2
            ctx.set_option("graph_halo", graph)
            for _ in range(5):
                T.atm_srk3(ctx, 720.0, 1)
            ctx.sync()
            ctx.download(got)
            out[graph] = (got, lib.halo_stats(ctx), ctx.get_option("graph_captures"),
                          ctx.get_option("graph_fallbacks"))
    bad = compare_states(out[1][0], out[0][0], rtol=0.0)
    assert not bad, bad[:6]
    assert out[1][1] == out[0][1]
    assert out[1][2] >= 1 and out[1][3] == 0, out[1][2:]
    got = d.local_state(0)
    with lib.Context(*d.n_local(0), st.L) as ctx:  # the default: RCCL steps run eagerly
        lib.setup_subdomain(ctx, d, 0)
        ctx.upload(got)
        lib.halo_rccl(ctx, 1, 0, lib.rccl_unique_id())
        for _ in range(3):
            T.atm_srk3(ctx, 720.0, 1)
        ctx.sync()
        assert ctx.get_option("graph_captures") == 0


def test_stub_latency_option(x1_2562):
    """option stub_latency_us (tools/rank_sim.py --latency-us): the stub's wire waits on the
    device; the values are unchanged and the step takes longer by about the waits"""
    import time
    st = state(x1_2562, 5, "random")
    d = decomp.Decomposition(st, 2)
    res = {}
    for lat in (0, 2000):
        loc = d.local_state(0)
        with lib.Context(*d.n_local(0), st.L) as ctx:
            lib.setup_subdomain(ctx, d, 0)
            lib.halo_stub(ctx)
            ctx.set_option("overlap", 0)
            ctx.set_option("graph_halo", 0)
            ctx.set_option("stub_latency_us", lat)
            assert ctx.get_option("stub_latency_us") == lat
            ctx.upload(loc)
            T.atm_srk3(ctx, 720.0, 1)
            ctx.sync()
            t = time.perf_counter()
            T.atm_srk3(ctx, 720.0, 1)
            ctx.sync()
            res[lat] = (time.perf_counter() - t, lib.halo_stats(ctx)[0])
            ctx.download(loc)
            res[lat] += (loc,)
    n_ex = res[0][1] / 2
    assert res[2000][0] - res[0][0] > 0.5 * n_ex * 2e-3, (res[0][:2], res[2000][:2])
    bad = compare_states(res[2000][2], res[0][2], rtol=0.0)
    assert not bad, bad[:6]
