"""tools/traffic_decomp.py: every dyn_tend kernel variant of a layout is matched
by its template arguments, and the tool fails loudly on a kernel it cannot place, on a kernel of the
layout missing from the counters, and on a negative refetch."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import traffic_decomp as TD  # noqa: E402

DIMS = (163842, 491520, 327680, 56)

# one kernel name per (launch kind, kernel) of each layout, as tools/pmc_kernels.py prints them
NAMES = {
    "r05": ["k_dyn_A<64, true, false>", "k_dyn_A<64, false, false>", "k_dyn_B<64, true, false, true, false, false>",
            "k_dyn_B<64, false, false, true, true, false>", "k_dyn_B<64, false, false, true, false, false>",
            "k_dyn_C12<64, false, 4>", "k_dyn_E<64, true, false, false, true>", "k_dyn_E<64, false, false, false, true>"],
    "r06": ["k_dyn_A<64, true, false>", "k_dyn_A<64, false, false>", "k_dyn_B<64, true, false, true, false, true>",
            "k_dyn_B<64, false, false, true, true, true>", "k_dyn_B<64, false, false, true, false, true>",
            "k_dyn_C12<64, false, 4>", "k_dyn_Et<true, false, true>", "k_dyn_Et<false, false, true>"],
    "r06ntu": ["k_dyn_A<64, true, false>", "k_dyn_E<64, false, false, false, true, true>",
               "k_dyn_B<64, true, false, true, false, true, true>", "k_dyn_A<64, false, false>",
               "k_dyn_B<64, false, false, true, true, false, false>", "k_dyn_C12<64, false, 4>",
               "k_dyn_E<64, true, false, false, true, true>", "k_dyn_E<64, false, false, false, true, false>"],
}


def _fixture(layout, scale=1.25):
    """counters at `scale` times each kernel's distinct bytes (FETCH_SIZE in KB, counted x2)"""
    lay = TD.LAYOUTS[layout]
    pmc = {n: {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0, "TCC_HIT_sum": 1.0, "TCC_MISS_sum": 1.0} for n in NAMES[layout]}
    # the distinct bytes of each kernel from a first pass at huge counters
    big = {n: {"FETCH_SIZE": 1e12, "WRITE_SIZE": 0.0} for n in NAMES[layout]}
    res = TD.decompose(big, layout, DIMS)
    for lk, d in res.items():
        for k in d["kernels"]:
            for n in k["names"]:
                pmc[n]["FETCH_SIZE"] = scale * k["compulsory_GB"] * 1e9 / 1e3 / 2
    assert set(lay) == set(res)
    return pmc


def _write(tmp_path, pmc):
    p = tmp_path / "kernels.txt"
    with open(p, "w") as f:
        for n, cs in pmc.items():
            f.write(n + "\n")
            for c, v in cs.items():
                f.write(f"    {c:40s} {v:16.6g}\n")
    return str(p)


@pytest.mark.parametrize("layout", ["r05", "r06", "r06ntu"])
def test_every_kernel_measured(tmp_path, layout):
    pmc = _fixture(layout)
    res = TD.decompose(TD.parse_kernels(_write(tmp_path, pmc)), layout, DIMS)
    for lk, d in res.items():
        assert len(d["kernels"]) == len(TD.LAYOUTS[layout][lk])
        for k in d["kernels"]:
            assert k["names"], (lk, k)
            assert k["refetch_GB"] == pytest.approx(0.25 * k["compulsory_GB"], rel=1e-4)
        assert d["measured_GB"] > d["compulsory_GB"]
    if layout == "r06":  # no per-edge flux scratch in the tiled layout
        assert all("X_F" not in d["arrays"] for d in res.values())


@pytest.mark.parametrize("layout", ["r05", "r06", "r06ntu"])
def test_fails_on_unmatched_missing_negative(tmp_path, layout):
    pmc = _fixture(layout)
    extra = dict(pmc, **{"k_dyn_B<64, false, true, true, false, true>": pmc[NAMES[layout][2]]})  # an MD B
    with pytest.raises(TD.DecompError, match="matches no kernel"):
        TD.decompose(extra, layout, DIMS)
    missing = {n: v for n, v in pmc.items() if n != NAMES[layout][6]}
    with pytest.raises(TD.DecompError, match="no k_dyn_E"):
        TD.decompose(missing, layout, DIMS)
    low = {n: dict(v) for n, v in pmc.items()}
    low[NAMES[layout][4]]["FETCH_SIZE"] *= 0.5
    with pytest.raises(TD.DecompError, match="negative refetch"):
        TD.decompose(low, layout, DIMS)


def test_cli_exit_status(tmp_path):
    import subprocess
    pmc = _fixture("r06")
    ok = subprocess.run([sys.executable, os.path.join(REPO, "tools", "traffic_decomp.py"), _write(tmp_path, pmc),
                         "--layout", "r06", "--round", "r06"], capture_output=True, text=True)
    assert ok.returncode == 0 and "traffic decomposition r06 (layout r06)" in ok.stdout
    bad = subprocess.run([sys.executable, os.path.join(REPO, "tools", "traffic_decomp.py"), _write(tmp_path, pmc),
                          "--layout", "r05"], capture_output=True, text=True)
    assert bad.returncode == 2 and "matches no kernel" in bad.stderr


def test_round5_counters_place_every_kernel():
    """the committed round-5 counters (profiles/r05/final_d) under the r05 layout: every B measured,
    no negative refetch (the round-5 table had neither)"""
    p = os.path.join(REPO, "profiles", "r05", "final_d", "pmc_kernels.txt")
    if not os.path.exists(p):
        pytest.skip("profiles/ not in this tree")
    res = TD.decompose(TD.parse_kernels(p), "r05", DIMS)
    for d in res.values():
        for k in d["kernels"]:
            assert k["refetch_GB"] >= 0.0
