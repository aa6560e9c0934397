"""bench.py's contract (one JSON line on stdout, the keys the driver reads) on the GPU, for
the single-GPU path and for the decomposed (RCCL halo) path at one rank -- the code the
multi-GPU run executes, short of the peers."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def run_bench(*args, timeout=110):
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--traffic", "off", *args], capture_output=True, text=True,
                       timeout=timeout, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, f"stdout must be ONE JSON line, got {len(lines)}: {p.stdout[:500]}"
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["single", "decompose"])
def test_bench_line(mode):
    d = run_bench(*(["--decompose"] if mode == "decompose" else []))
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0 and d["ms_per_step"] > 0
    assert d["unit"] == "Mcell-columns/s" and d["dtype"] == "f64" and d["cpu_baseline"] is None
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and 0 < r["frac"] < 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    if mode == "decompose":
        assert d["scaling"] == "strong" and d["config"]["parallelism"] == "decomposed1"
        assert d["halo"]["exchanges_per_step"] > 0 and d["halo"]["ghost_frac"] == [0.0, 0.0, 0.0]
    else:
        assert d["scaling"] == "weak" and d["config"]["parallelism"] == "single-gpu"


@pytest.mark.gpu
def test_bench_multirank_flow_socket():
    """--gpus 2 --halo socket: bench.py spawns two rank processes that share the one GPU,
    meet over the TCP rendezvous, split the mesh and exchange halos over the host-staged
    socket transport -- the multi-rank flow of the driver's N-GPU run (rank spawning,
    rendezvous, decomposition, max-over-ranks timing, one JSON line), RCCL aside"""
    d = run_bench("--gpus", "2", "--halo", "socket", "--ncells", "2562")
    assert KEYS <= set(d)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    assert d["halo"]["transport"].startswith("socket") and d["halo"]["exchanges_per_step"] > 0
    assert all(0 < g < 0.5 for g in d["halo"]["ghost_frac"][:1])


@pytest.mark.gpu
def test_bench_line_transport():
    """--transport: the MPAS solver and the scalar transport inside the timed step"""
    d = run_bench("--transport")
    assert KEYS <= set(d)
    assert d["config"]["physics"] == 1 and d["config"]["transport"] == 1
    assert "atm_advance_scalars_mono" in d["tasks"] and d["tasks"]["atm_advance_scalars_mono"]["launches_per_step"] == 1
    assert d["tasks"]["atm_advance_acoustic_step_work"]["launches_per_step"] == 4


@pytest.mark.gpu
def test_bench_roofline_is_dyn_tend_with_live_traffic():
    """the roofline names the north-star task (dyn_tend: rk0 + 2 rk>0 launches per step),
    and its traffic comes from rocprofv3 FETCH_SIZE / WRITE_SIZE passes of the same
    workload run by bench.py itself (x1.40962 keeps the passes short)"""
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--ncells", "40962"], capture_output=True, text=True, timeout=300,
                       cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip())
    r = d["roofline"]
    assert r["kernel"] == "atm_compute_dyn_tend_work" and r["launches_per_step"] == 3
    # (options fusecopy, defer4, ntu and vdyn tag the launches whose read / write sets they change;
    # ntu: stage 0 and 1 form no dead tendency, the deferred del4 goes to stage 2 with v; -A: A ran
    # in a combined launch on small grids)
    tags = sorted(t.replace("-A]", "]") for t in r["variants"])
    assert tags == ["[rk0+copy+d4o+ntu]", "[rk>0+d4i+v]", "[rk>0+ntu]"], tags
    assert sum(v["launches_per_step"] for v in r["variants"].values()) == 3
    assert r["traffic"] is not None, r["traffic_source"]
    # measured traffic cannot be below the distinct arrays the task must touch (minus the
    # 2-D mesh rows, which may stay in cache), nor absurdly above
    assert 0.5 * r["b_alg_per_launch_GB"] < r["traffic"] < 10 * r["b_alg_per_launch_GB"]


@pytest.mark.gpu
def test_bench_8rank_headline_socket(tmp_path):
    """the driver's 8-GPU flow at the headline size, rehearsed on the one
    GPU -- bench.py --gpus 8 spawns 8 rank processes, each splits x1.163842 x 56 8 ways
    (the split the 8-GPU run uses), builds its pack / unpack address tables and exchanges
    halos (host-staged socket transport in RCCL's place).  The owned rows of the 8 ranks,
    assembled by global id, equal one undecomposed context bit for bit (exact mode; per-row
    64-bit fingerprints of every fp64 field, bench.py dump_rows), and every rank made the
    exchanges per step the in-process loopback split makes (x1.2562, 2 parts: the count is
    the launch sequence's, not the mesh's)"""
    import numpy as np
    sys.path.insert(0, REPO)
    import bench
    from mpasdyn import decomp, lib
    from mpasdyn import tasks as T
    from mpasdyn.registry import FIELDS

    common = ("--steps", "1", "--warmup", "1", "--exact", "1", "--ncells", "163842")
    d8 = run_bench("--gpus", "8", "--halo", "socket", *common, "--dump", str(tmp_path / "r8"), timeout=150)
    assert d8["n_gpus"] == 8 and d8["config"]["parallelism"] == "decomposed8" and d8["value"] > 0
    run_bench(*common, "--dump", str(tmp_path / "r1"), timeout=100)
    one = np.load(tmp_path / "r1" / "rank0.npz")
    names = [f.name for f in FIELDS if f.entity is not None and f.dtype == np.float64]
    seen = {k: np.zeros(len(one[f"gid_{k}"]), dtype=bool) for k in ("cell", "edge", "vertex")}
    ex = []
    for r in range(8):
        part = np.load(tmp_path / "r8" / f"rank{r}.npz")
        assert int(part["steps"]) == int(one["steps"]) == 2 and int(part["world"]) == 8
        ex.append(int(part["exchanges"]))
        for k in seen:
            seen[k][part[f"gid_{k}"]] = True
        bad = [n for n in names
               if not np.array_equal(part[n], one[n][part["gid_" + next(f.entity for f in FIELDS if f.name == n)]])]
        assert not bad, f"rank {r}: owned rows differ from the single context in {bad[:8]}"
    assert all(v.all() for v in seen.values())  # (the 8 ranks own every entity)
    # the exchanges of the same two steps in the in-process loopback split
    m, st = bench.build_inputs(2562, 56)
    dec = decomp.Decomposition(st, 2)
    ctxs = [lib.Context(*dec.n_local(r), 56) for r in range(2)]
    try:
        import threading
        for r, c in enumerate(ctxs):
            c.set_option("exact", 1)
            lib.setup_subdomain(c, dec, r)
            bench.upload_inputs(c, dec.local_state(r))
        lib.halo_loopback(ctxs)
        th = [threading.Thread(target=lambda c=c: [T.atm_srk3(c, bench.dt_for(2562), 1) for _ in range(2)])
              for c in ctxs]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        for c in ctxs:
            c.sync()
        loop = lib.halo_stats(ctxs[0])[0]
    finally:
        for c in ctxs:
            c.close()
    assert ex == [loop] * 8, (ex, loop)
