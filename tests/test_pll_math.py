"""The PLL's certified fast sin/cos/atan2 (csrc/pll_math.h) against glibc, on the host.

Whenever the fast path claims a float result it must equal float(glibc(x)) -- the value the
reference's PLL feeds back into itself (src/filter.cpp:161-170).  The full sweep (every float
in +-[1, 8.5e6], the whole PLL argument range) was run with tools/check_pll_math.cpp; this
test re-checks a strided subset plus random atan2 pairs in CI time."""
import os
import subprocess

import pytest

from conftest import REPO


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pllm") / "check_pll_math")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-o", exe,
                    os.path.join(REPO, "tools", "check_pll_math.cpp")], check=True)
    return exe


@pytest.mark.parametrize("lo,hi,stride", [("1e-30", "1", "401"), ("1", "8.5e6", "29"),
                                          ("8.5e6", "1e9", "7")])
def test_sincos_fast_path_matches_glibc(checker, lo, hi, stride):
    r = subprocess.run([checker, "sincos", lo, hi, stride], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout
    assert "mismatches=0" in r.stdout


def test_atan2_fast_path_matches_glibc(checker):
    r = subprocess.run([checker, "atan2", "20000000", "3"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout
    assert "mismatches=0" in r.stdout
