"""K1's accept test screens attempts in float and falls back to the exact double test near the
unit circle (df_rng.hpp polar_screen). On the host, with the product header itself, it must take
the same decision as the exact test for every attempt (2e7 per seed; ~600 land in the band)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


def test_float_screened_accept_equals_exact(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = tmp_path / "check_polar_accept"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17",
                    "-I" + os.path.join(ROOT, "digital-filtering_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "check_polar_accept.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "5000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
