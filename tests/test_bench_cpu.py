"""bench.py host logic on the CPU: the --gpus N launcher (N rank processes with the
rendezvous environment, started before any GPU call), the WORLD_SIZE check, and the
per-task roofline aggregation (one Regent task = all its timing variants)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=120, cwd=REPO, env=e)


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_starts_n_ranks(n):
    p = _run(["--gpus", str(n), "--dry-run"])
    assert p.returncode == 0, p.stderr
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.strip()]
    lines += [json.loads(x) for x in p.stderr.splitlines() if x.startswith("{")]
    assert sorted(d["rank"] for d in lines) == list(range(n))
    assert all(d["world_size"] == n and d["gpus"] == n and d["local_rank"] == d["rank"] for d in lines)
    masters = {d["master"] for d in lines}
    assert len(masters) == 1 and masters.pop().startswith("127.0.0.1:")


def test_launcher_single_rank_runs_in_process():
    p = _run(["--dry-run"])
    assert p.returncode == 0, p.stderr
    d = json.loads(p.stdout.strip())
    assert d == {**d, "rank": 0, "world_size": 1, "gpus": 1}


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr


def test_launcher_propagates_rank_failure():
    # an unknown option makes every rank exit 2 (argparse) -> the launcher exits non-zero
    p = _run(["--gpus", "2", "--no-such-flag"])
    assert p.returncode != 0


def test_task_table_aggregates_variants():
    import bench
    from mpasdyn import roofline
    dims = (163842, 491520, 327680, 56)
    # two profiled steps: dyn_tend 1 rk0 + 2 rk>0 launches per step, acoustic 3 + 4
    rep = {"atm_compute_dyn_tend_work[rk0]": (2, 2 * 2.7), "atm_compute_dyn_tend_work[rk>0]": (4, 4 * 1.3),
           "atm_advance_acoustic_step_work[ss0]": (6, 6 * 0.35), "atm_advance_acoustic_step_work[ss>0]": (8, 8 * 0.44),
           "atm_divergence_damping_3d": (14, 14 * 0.14)}
    t = bench.task_table(rep, dims, 2, physics=False)
    dyn = t["atm_compute_dyn_tend_work"]
    b0 = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=0)
    b1 = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=1)
    assert dyn["launches_per_step"] == 3 and abs(dyn["ms_per_step"] - (2.7 + 2 * 1.3)) < 1e-9
    gbs = (b0 + 2 * b1) / ((2.7 + 2 * 1.3) * 1e-3) / 1e9
    assert abs(dyn["GBs"] - gbs) < 0.1 and abs(dyn["frac"] - gbs / 8000.0) < 1e-4
    assert set(dyn["variants"]) == {"[rk0]", "[rk>0]"}
    ac = t["atm_advance_acoustic_step_work"]
    a0 = roofline.b_alg("atm_advance_acoustic_step_work", dims, small_step=0)
    a1 = roofline.b_alg("atm_advance_acoustic_step_work", dims, small_step=1)
    assert a0 < a1  # the first substep reads four columns fewer
    assert abs(ac["b_alg_GB_per_step"] - (3 * a0 + 4 * a1) / 1e9) < 1e-3
    # the task with the most device time per step is dyn_tend, not the 7-launch acoustic task
    assert max(t, key=lambda k: t[k]["ms_per_step"]) == "atm_compute_dyn_tend_work"


def test_pmc_kernel_map_covers_fused_launches():
    """every kernel of the fused schedules is attributed (dyn_tend's combined rk 0 D/E
    launch to dyn_tend), and the standalone setup run that calibrates WRITE_SIZE is
    removed from the per-step bytes"""
    from mpasdyn import pmc
    assert pmc.task_of("k_dyn_DE<64, true>") == "atm_compute_dyn_tend_work[rk0]"
    assert pmc.task_of("k_dyn_B<64, false, 2>") == "atm_compute_dyn_tend_work[rk>0]"
    assert pmc.task_of("k_setup_vi<64>") == "atm_rk_integration_setup"
    assert pmc.task_of("k_hf_e_vi") == "hfuse"
    assert pmc.task_of("k_acoustic<64, false, true, true, false, 2, true, true>") == "atm_advance_acoustic_step_work"
    L, nc, ne = 56, 40962, 3 * (40962 - 2)
    payload = (7 * nc + 2 * ne) * 8 * L
    w = {"k_copy64": (2 * payload / 1024.0 / 0.875, 2), "k_dyn_DE<64, true>": (100.0, 1)}
    assert abs(pmc.write_factor(w, nc, ne, L) - 0.875) < 1e-12
    d = pmc.drop_calibration(w)
    assert d["k_copy64"] == (payload / 1024.0 / 0.875, 1) and d["k_dyn_DE<64, true>"] == (100.0, 1)
    assert "k_copy64" not in pmc.drop_calibration({"k_copy64": (5.0, 1)})


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_rendezvous_without_torch(n):
    """--dry-run runs one round of the host rendezvous (mpasdyn/rendezvous.py): rank 0's
    unique-id bytes reach every rank, the max over ranks is world - 1 everywhere, and no
    rank imported torch (the bench's process holds one HIP runtime, the library's)"""
    p = _run(["--gpus", str(n), "--dry-run"])
    assert p.returncode == 0, p.stderr
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.strip()]
    lines += [json.loads(x) for x in p.stderr.splitlines() if x.startswith("{")]
    assert len(lines) == n
    assert all(d["bcast"] == "uid-from-rank-0" and d["max_rank"] == n - 1 for d in lines)
    assert not any(d["torch_loaded"] for d in lines)


def test_single_rank_dry_run_without_torch():
    p = _run(["--dry-run"])
    assert p.returncode == 0 and json.loads(p.stdout.strip())["torch_loaded"] is False


def test_free_port_range():
    import bench
    base = bench.free_port_range(4)
    assert 1024 < base < 65535 - 4


def test_rendezvous_in_threads():
    """the rendezvous' collectives at world 4, ranks as threads of one process"""
    import threading
    from mpasdyn.rendezvous import Rendezvous
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = {}

    def rank(r):
        rv = Rendezvous(r, 4, "127.0.0.1", port, timeout=30)
        b = rv.bcast(b"\x01\x02" * 64 if r == 0 else None)
        m = rv.allreduce_max(10.0 * r - r * r)  # max at r = 3 (21), not at the last rank
        rv.barrier()
        rv.close()
        out[r] = (b, m)
    th = [threading.Thread(target=rank, args=(r,)) for r in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert sorted(out) == [0, 1, 2, 3]
    assert all(b == b"\x01\x02" * 64 and m == 21.0 for b, m in out.values())


def test_roofline_fusecopy_moves_the_edge_copies():
    """option fusecopy: setup's ru_save / u_2 copies counted in stage 0's dyn_tend launch;
    the step's B_alg loses exactly the second read of ru and u"""
    from mpasdyn import roofline
    dims = (163842, 491520, 327680, 56)
    e3 = 8 * 491520 * 56
    a = roofline.b_alg_step(dims, 1, 0, 0, True, True, True, False)
    b = roofline.b_alg_step(dims, 1, 0, 0, True, True, True, True)
    assert a - b == 2 * e3
    s0 = roofline.b_alg("atm_rk_integration_setup", dims, fused=True)
    s1 = roofline.b_alg("atm_rk_integration_setup", dims, fused=True, copy=True)
    d0 = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=0)
    d1 = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=0, copy=True)
    assert s0 - s1 == 4 * e3 and d1 - d0 == 2 * e3
    # the MPAS forms (round 5: srk3 applies fusecopy under every physics mode)
    for physics in (1, 2):
        a = roofline.b_alg_step(dims, 1, physics, 0, False, True, False, False)
        b = roofline.b_alg_step(dims, 1, physics, 0, False, True, False, True)
        assert a - b == 2 * e3


def test_roofline_defer4_and_vdyn_accounting():
    """option defer4: stage 0's dead tend_u store is taken out of that launch's B_alg (no
    credit for bytes not moved), the receiving launch gets none for what it adds; option
    vdyn: stage 2's launch is credited the v it stores; bench.py reads the variant tags"""
    import bench
    from mpasdyn import roofline
    dims = (163842, 491520, 327680, 56)
    e3 = 8 * 491520 * 56
    d0 = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=0, copy=True)
    d0o = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=0, copy=True, defer_out=True)
    assert d0 - d0o == e3
    d1 = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=1)
    d1v = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=1, store_v=True)
    assert d1v - d1 == e3
    a = roofline.b_alg_step(dims, 1, 0, 0, True, True, True, True, False)
    b = roofline.b_alg_step(dims, 1, 0, 0, True, True, True, True, True)
    assert a - b == e3
    rep = {"atm_compute_dyn_tend_work[rk0+copy+d4o]": (2, 4.4), "atm_compute_dyn_tend_work[rk>0+d4i]": (2, 2.8),
           "atm_compute_dyn_tend_work[rk>0+v-A]": (2, 2.2)}
    t = bench.task_table(rep, dims, 2, physics=False)["atm_compute_dyn_tend_work"]
    na = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=1, store_v=True, noA=True)
    assert abs(t["b_alg_GB_per_step"] - (d0o + d1 + na) / 1e9) < 1e-3
    assert set(t["variants"]) == {"[rk0+copy+d4o]", "[rk>0+d4i]", "[rk>0+v-A]"}
    # the fraction without the fusecopy bytes: the rk_step 0 launch's
    # ru_save / u_2 stores out, nothing else
    d0x = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=0, defer_out=True)
    assert d0o - d0x == 2 * e3
    assert t["variants"]["[rk0+copy+d4o]"]["b_alg_GB_excl_fusecopy"] == round(d0x / 1e9, 4)
    want = (d0x + d1 + na) / 1e9 / (t["ms_per_step"] * 1e-3) / bench.HBM_PEAK_GBS
    assert abs(bench.frac_excl_copy(t) - want) < 2e-4


def test_roofline_acoustic_rtheta_pp_old_accounting():
    """option fusedamp: only the step's last acoustic launch stores rtheta_pp_old (the fused
    damping reads the stored div), so the other six fused launches are credited no
    rtheta_pp_old write; the library tags them "-old" and bench.py reads the tag"""
    import bench
    from mpasdyn import roofline
    dims = (163842, 491520, 327680, 56)
    c3 = 8 * 163842 * 56
    a = roofline.b_alg("atm_advance_acoustic_step_work", dims, small_step=1, damp=True)
    b = roofline.b_alg("atm_advance_acoustic_step_work", dims, small_step=1, damp=True, wold=False)
    assert a - b == c3
    for sml in (True, False):
        fused = roofline.b_alg_step(dims, 1, 0, 0, True, True, sml, True, True)
        sched = roofline.step_schedule(1, 0, 0, True, True, sml, True, True)
        n_ac = sum(n for t, kw, n in sched if t == "atm_advance_acoustic_step_work")
        n_old = sum(n for t, kw, n in sched if t == "atm_advance_acoustic_step_work" and kw.get("wold", True))
        assert (n_ac, n_old) == (7, 1)
        # against the same schedule with every launch credited the write
        full = sum(roofline.b_alg(t, dims, **{k: v for k, v in kw.items() if k != "wold"}) * n for t, kw, n in sched)
        assert full - fused == 6 * c3
    rep = {"atm_advance_acoustic_step_work[ss>0+damp-old]": (3, 1.5), "atm_advance_acoustic_step_work[ss>0+damp]": (1, 0.5)}
    t = bench.task_table(rep, dims, 1, physics=False)["atm_advance_acoustic_step_work"]
    assert abs(t["b_alg_GB_per_step"] - (3 * b + a) / 1e9) < 1e-3


def test_roofline_smlsum_accounting():
    """option smlsum: set_smlstep's zb_cell / zb3_cell / u_tend / edge-sign reads counted once per
    step (the flux task) instead of in each of the three fused acoustic launches; the flux task
    also reads the cell's edge list, which the acoustic launches share; bench.py reads the tags"""
    import bench
    from mpasdyn import roofline
    dims = (163842, 491520, 327680, 56)
    fb = lambda n: roofline.field_bytes(n, *dims)  # noqa: E731
    a = roofline.b_alg_step(dims, 1, 0, 0, True, True, True, True, True, False)
    b = roofline.b_alg_step(dims, 1, 0, 0, True, True, True, True, True, True)
    kw = dict(small_step=0, damp=True, sml=True, wold=False)
    d_ac = roofline.b_alg("atm_advance_acoustic_step_work", dims, **kw) - \
        roofline.b_alg("atm_advance_acoustic_step_work", dims, smls=True, **kw)
    flux = roofline.b_alg("atm_set_smlstep_pert_variables_work", dims, part="flux")
    dd = fb("rw") + fb("rw_save")  # (X_Dd = rw_save - rw, formed by the flux task, read by all 7 launches)
    assert flux - d_ac == fb("nEdgesOnCell") + fb("edgesOnCell") + dd  # (the acoustic launch reads the lists anyway)
    assert d_ac > fb("u_tend") + fb("edgesOnCell_sign")  # (+ the zb_cell / zb3_cell components)
    assert a - b == 3 * d_ac - flux + 7 * dd
    rep = {"atm_set_smlstep_pert_variables_work[flux]": (1, 0.2),
           "atm_advance_acoustic_step_work[ss0+smlS+damp-old]": (2, 1.2)}
    t = bench.task_table(rep, dims, 1, physics=False, ddx=True)
    assert abs(t["atm_set_smlstep_pert_variables_work"]["b_alg_GB_per_step"] - flux / 1e9) < 1e-3
    ac = roofline.b_alg("atm_advance_acoustic_step_work", dims, small_step=0, damp=True, sml=True, smls=True,
                        wold=False, ddx=True)
    assert ac == roofline.b_alg("atm_advance_acoustic_step_work", dims, small_step=0, damp=True, sml=True, smls=True,
                                wold=False) - dd
    assert abs(t["atm_advance_acoustic_step_work"]["b_alg_GB_per_step"] - 2 * ac / 1e9) < 1e-3


def test_b_alg_ntu():
    """option ntu: the rk_step 0 launch takes no credit for the arrays only its dead tend_u read"""
    from mpasdyn import roofline
    dims = (163842, 491520, 327680, 56)
    a = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=0, copy=True, defer_out=True)
    b = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=0, copy=True, defer_out=True, ntu=True)
    e3, c3 = 8 * dims[1] * dims[3], 8 * dims[0] * dims[3]
    assert a - b >= 2 * e3 + 2 * c3  # pv_edge, tend_ru_physics, ke, w (+ their mesh rows)
    r, w = roofline._sets("atm_compute_dyn_tend_work", rk_step=0, defer_out=True, ntu=True)
    assert "pv_edge" not in r and "ke" not in r and "u" in r and "theta_m" in r
    assert "tend_theta" not in w and "tend_theta_euler" in w and "w" in w and "tend_u_euler" in w
    r1, w1 = roofline._sets("atm_compute_dyn_tend_work", rk_step=1, ntu=True)
    assert set(w1) == {"w"} and "ru" in r1 and "tend_w_euler" in r1 and "theta_m" not in r1
    # under the MPAS forms the option changes nothing (the tendencies are live)
    assert roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=0, ntu=True, physics=2) == \
        roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=0, physics=2)
    s0 = roofline.b_alg_step(dims, 1, 0, 0, True, True, True, True, True, True, False)
    s1 = roofline.b_alg_step(dims, 1, 0, 0, True, True, True, True, True, True, True)
    b1 = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=1)
    c1 = roofline.b_alg("atm_compute_dyn_tend_work", dims, rk_step=1, ntu=True)
    sd = roofline.b_alg("atm_compute_solve_diagnostics", dims)
    sl = roofline.b_alg("atm_compute_solve_diagnostics", dims, live=True)
    # (+ stage 0's dead solve_diagnostics, the dead stores and reads of stage 1's, and the acoustic
    # state the last substep of stages 0 and 1 leaves unstored)
    ac = roofline.b_alg("atm_advance_acoustic_step_work", dims, small_step=1, damp=True, wold=False, ddx=True)
    an = roofline.b_alg("atm_advance_acoustic_step_work", dims, small_step=1, damp=True, wold=False, ddx=True, nst=True)
    assert ac - an == 5 * c3  # rho_pp, rtheta_pp, rw_p, wwAvg; the wwAvg read
    # (+ stage 0's b_tri / c_tri, which stage 1's vert_imp rewrites, and the substep finish's rho_zz copy,
    # the identity in atm_srk3: a read and a write)
    assert s0 - s1 == (a - b) + (b1 - c1) + sd + (sd - sl) + 2 * (ac - an) + 2 * c3 + 2 * c3
    r, w = roofline._sets("atm_compute_solve_diagnostics", live=True)
    assert set(w) == {"ke", "pv_edge", "pv_vertex"} and "h" not in r and "u" in r
    assert sd - sl >= 2 * e3 + 3 * c3  # h_edge, ke_edge, divergence, h (+ vorticity at the vertices)
