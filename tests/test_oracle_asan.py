"""SURVEY §5 (sanitizers): the CPU oracle restatement run under AddressSanitizer and
UndefinedBehaviorSanitizer (oracle/asan_driver.c: every task, both rk_step and small_step
branches, the two srk3 drivers, the MPAS solver and the transport, on small states with
random in-policy connectivity, at 7 and 26 levels and the degenerate 1 and 2).  Any out-of-bounds access, leak or UB aborts the build
target with a non-zero status."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no C compiler")
def test_oracle_clean_under_asan_ubsan():
    p = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan-run"], capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    assert p.stdout.count("ran clean") == 4  # 7 and 26 levels, and the degenerate 1 and 2
