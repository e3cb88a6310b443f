"""Fortran coupling: include/digital_filtering.f90 compiled with amdflang
into examples/fortran-main, the reference's Fortran driver shape
(digital-filtering-fortran/test/fortran-main.f90) on libdfamd.so.

CPU: host-only handles through the Fortran module reproduce the reference's golden
setup rows and half-widths (the bind(C) struct layout is checked by the module
itself against df_config_sizeof). GPU: the Fortran path reproduces the golden
fields, matches the Python/C path bit for bit (same library), and df_gather_field
injects u' into a caller-owned device array exactly.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import dfamd
from conftest import GOLDEN, ROOT

EXE = os.path.join(ROOT, "examples", "fortran-main")
TOL = 1e-6


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE):
        if not shutil.which("amdflang"):
            pytest.skip("amdflang not installed and examples/fortran-main not prebuilt")
        subprocess.run(["make", "-C", os.path.join(ROOT, "examples"), EXE], check=True, capture_output=True)
    return EXE


def run(exe, *args):
    return subprocess.run([exe, *map(str, args)], cwd=ROOT, capture_output=True, text=True, timeout=300)


def read_setup(path):
    raw = open(path, "rb").read()
    Ny, Nz = np.frombuffer(raw, np.int32, 2)
    u_tau, tau_w = np.frombuffer(raw, np.float64, 2, offset=8)
    off = 24
    rows = np.frombuffer(raw, np.float64, 5 * Ny, offset=off).reshape(5, Ny)
    off += 40 * Ny
    hw = np.frombuffer(raw, np.int32, 6 * Ny * Nz, offset=off).reshape(6, Ny, Nz)
    return int(Ny), int(Nz), u_tau, tau_w, rows, hw


def rel_err(a, b):
    rms = np.sqrt((b * b).mean(axis=-1, keepdims=True))
    scale = np.maximum(np.abs(b), rms)
    diff = np.abs(a - b)
    return np.where(scale > 0, diff / np.where(scale > 0, scale, 1.0), np.where(diff > 0, np.inf, 0.0))


@pytest.mark.parametrize("name", ["native_s42", "c1_s42", "ramp256_s1234", "ragged_s7"])
def test_fortran_host_setup_matches_reference(exe, tmp_path, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    if name.startswith("native"):
        plane, dims = 0, (0, 0, 0, 0)
        py = dfamd.DigitalFilter(device=-1, seed=1)
    else:
        dims = (int(g["Ny"]), int(g["Nz"]), int(g["N_min"]), int(g["N_max"]))
        plane = 1
        py = dfamd.DigitalFilter(device=-1, seed=1, plane="synthetic", Ny=dims[0], Nz=dims[1], N_min=dims[2],
                                 N_max=dims[3])
    out = tmp_path / "setup.bin"
    r = run(exe, "host", plane, *dims, out)
    assert r.returncode == 0, r.stdout + r.stderr
    Ny, Nz, u_tau, tau_w, rows, hw = read_setup(out)
    assert (Ny, Nz) == (py.Ny, py.Nz)
    assert u_tau == py.scalar("u_tau") and tau_w == py.scalar("tau_w")
    for i, k in enumerate(("R11", "R21", "R22", "R33")):
        assert np.array_equal(rows[i], g["row_" + k]), k
    assert np.array_equal(rows[4], py.row("yc"))
    for c, n in enumerate("uvw"):
        assert np.array_equal(hw[2 * c][:, 0], g["Ny_" + n]), n
        assert np.array_equal(hw[2 * c + 1][:, 0], g["Nz_" + n]), n
        assert np.array_equal(hw[2 * c], py.halfwidths(c, "y"))
        assert np.array_equal(hw[2 * c + 1], py.halfwidths(c, "z"))


def test_fortran_errors_stop_loudly(exe, tmp_path):
    r = run(exe, "host", 1, 1, 4, 2, 4, tmp_path / "x.bin")  # a 1-row synthetic plane is invalid
    assert r.returncode != 0
    assert "DIGITAL_FILTERING: create_digital_filter" in r.stdout and "synthetic" in r.stdout


# ---------------------------------------------------------------- GPU

def read_run(path, Ny, Nz):
    raw = open(path, "rb").read()
    ny, nz = np.frombuffer(raw, np.int32, 2)
    assert (ny, nz) == (Ny, Nz)
    state = int(np.frombuffer(raw, np.uint64, 1, offset=8)[0])
    flag = int(np.frombuffer(raw, np.int32, 1, offset=16)[0])
    saved = float(np.frombuffer(raw, np.float64, 1, offset=20)[0])
    f = np.frombuffer(raw, np.float64, 6 * Ny * Nz, offset=28).reshape(6, Ny, Nz)
    return (state, flag, saved), dict(zip(("u", "v", "w", "T", "rho", "filt_old_u"), f))


@pytest.mark.gpu
@pytest.mark.parametrize("name,steps", [("c1_s42", 3), ("ragged_s7", 2)])
def test_fortran_filter_matches_golden_and_c_path(exe, tmp_path, name, steps):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    Ny, Nz, a, b = int(g["Ny"]), int(g["Nz"]), int(g["N_min"]), int(g["N_max"])
    st = (int(g["start_state"]), int(g["start_saved_flag"]), float(g["start_saved"]))
    signed = st[0] - (1 << 64) if st[0] >= 1 << 63 else st[0]
    out = tmp_path / "run.bin"
    r = run(exe, "run", 1, Ny, Nz, a, b, 0, steps, repr(float(g["dt"])), out, signed, st[1], repr(st[2]))
    assert r.returncode == 0, r.stdout + r.stderr
    state, fields = read_run(out, Ny, Nz)
    for k in ("u", "v", "w", "T", "rho"):  # the reference's own output (tests/golden, gen_golden.py)
        assert np.array_equal(fields[k], g[f"s{steps}_{k}"]), (k, float(rel_err(fields[k], g[f"s{steps}_{k}"]).max()))
    py = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=a, N_max=b, device=0, resume=st)
    for _ in range(steps):
        py.filter(float(g["dt"]))
    assert state == py.rng_state()
    for k in ("u", "v", "w", "T", "rho"):
        assert np.array_equal(fields[k], py.field(k)), k
    assert np.array_equal(fields["filt_old_u"], py.field("filt_old_u"))


@pytest.mark.gpu
def test_fortran_device_gather_injects_fluctuations(exe, tmp_path):
    out = tmp_path / "gather.bin"
    r = run(exe, "gather", 1, 96, 70, 2, 12, 9, out)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(out, "rb").read()
    Ny, Nz = np.frombuffer(raw, np.int32, 2)
    n = int(Ny) * int(Nz)
    u, base, got = np.frombuffer(raw, np.float64, 3 * n, offset=8).reshape(3, n)
    assert np.any(u != 0)
    assert np.array_equal(got, base + u[::-1])


@pytest.mark.gpu
def test_fortran_reference_driver_flow(exe):
    # fortran-main.f90 with no arguments: native plane, random_device seed, filter(1e-8)
    r = run(exe)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "plane 510 x 400" in r.stdout
