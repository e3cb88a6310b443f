"""Host code of libdfamd (df_capi.cpp, df_setup.cpp) under AddressSanitizer + UBSan.

The two host translation units are rebuilt with `-Xarch_host -fsanitize=address,undefined`
(device code unchanged: the prebuilt kernel object is linked as is) into a driver that
creates host-only handles (device = -1: no GPU) of every plane kind — the reference's own
grid, synthetic and ragged planes in both coefficient modes, caller-vertex grids with
per-cell half-widths, z-strip planning — calls every host accessor and walks the error
paths (tests/cpp/host_sanitize.cpp). Any sanitizer report or failed check fails the test.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "digital-filtering_amd")
HIPCC = "/opt/rocm/bin/hipcc"
KOBJ = os.path.join(PKG, "build", "df_kernels.o")


@pytest.mark.skipif(not os.path.exists(HIPCC) or not os.path.exists(KOBJ), reason="needs hipcc and a built libdfamd")
def test_host_code_clean_under_asan_ubsan(tmp_path):
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-omit-frame-pointer"]
    common = ["-std=c++17", "-O1", "-g", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950",
              "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc")]
    capi, setup, drv, exe = (str(tmp_path / n) for n in ("capi.o", "setup.o", "drv.o", "host_sanitize"))
    run = lambda cmd: subprocess.run(cmd, check=True, capture_output=True, text=True)  # noqa: E731
    run([HIPCC, *common, *san, "-x", "hip", "-c", os.path.join(PKG, "csrc", "df_capi.cpp"), "-o", capi])
    run([HIPCC, *common, *san, "-c", os.path.join(PKG, "csrc", "df_setup.cpp"), "-o", setup])
    # the driver is plain C++ over df_c.h: host compiler and host link (the HIP objects carry their
    # device code; libamdhip64 registers it)
    host_san = ["-fsanitize=address", "-fsanitize=undefined", "-fno-omit-frame-pointer"]
    run(["g++", "-std=c++17", "-O1", "-g", "-I" + os.path.join(ROOT, "include"), *host_san,
         "-c", os.path.join(ROOT, "tests", "cpp", "host_sanitize.cpp"), "-o", drv])
    run(["g++", *host_san, drv, capi, setup, KOBJ, "-L/opt/rocm/lib", "-lamdhip64", "-lrccl",
         "-Wl,-rpath,/opt/rocm/lib", "-o", exe])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    data = os.path.join(PKG, "data")
    out = subprocess.run([exe, os.path.join(data, "RST.dat"), os.path.join(data, "line.dat")],
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "host sanitize: ok" in out.stdout
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr
    shutil.rmtree(tmp_path, ignore_errors=True)
