"""The polar transform's table-driven log (df_rng.hpp log_r2, used by K3 on the GPU) against glibc's
log, which the reference's libstdc++ normal_distribution calls (random.tcc:1828): on the host, with
the product header itself, over r2 values of the pcg32 polar stream, uniform (0, 1], arguments within
2^-20 below 1 and tiny ones - at most 1 ulp apart (the device library's log it replaces is also within
1 ulp). And glibc_log (df_rng.hpp, K3's default since round 2), glibc 2.35's own algorithm on its own
constants: bit-identical to the host's log on every argument, so the GPU normals equal the reference's
bit for bit (tests/test_gpu_parity.py)."""
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
    assert r.stdout.split()[-1] == "0", r.stdout  # glibc_log_mismatch


def test_glibc_log_table_matches_this_libm(tmp_path):
    # the committed constants are the ones in this image's libm (tools/gen_glibc_log_table.py)
    libm = "/lib/x86_64-linux-gnu/libm.so.6"
    if not os.path.exists(libm):
        pytest.skip("no glibc libm at " + libm)
    out = tmp_path / "t.h"
    subprocess.run(["python3", os.path.join(ROOT, "tools", "gen_glibc_log_table.py"), libm, str(out)], check=True,
                   capture_output=True)
    ref = os.path.join(ROOT, "digital-filtering_amd", "csrc", "glibc_log_table.h")
    assert out.read_text() == open(ref).read()
