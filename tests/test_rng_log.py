"""The polar transform's table-driven log (df_rng.hpp log_r2, used by K3 on the GPU) against glibc's
log, which the reference's libstdc++ normal_distribution calls (random.tcc:1828): on the host, with
the product header itself, over r2 values of the pcg32 polar stream, uniform (0, 1], arguments within
2^-20 below 1 and tiny ones - at most 1 ulp apart (the device library's log it replaces is also within
1 ulp; GPU normals are checked within 2 ulp of the reference's in tests/test_gpu_parity.py)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


def test_log_r2_within_one_ulp_of_glibc(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = tmp_path / "check_log_r2"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17",
                    "-I" + os.path.join(ROOT, "digital-filtering_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "check_log_r2.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "3000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("max_ulp ") and int(r.stdout.split()[1]) <= 1, r.stdout
