"""GPU tests of the drop-in surfaces: the reference driver rebuilt on include/df.hpp
(examples/cpp-test), the get_rms() statistics path, the CSV writer, and the
SURVEY §4 variance invariant."""
import os
import subprocess

import numpy as np
import pytest

import dfamd
import oracle as O
from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
FIELDS = ("u", "v", "w", "T", "rho")
EXE = os.path.join(ROOT, "examples", "cpp-test")


def rel_err(a, b):
    rms = np.sqrt((b * b).mean(axis=-1, keepdims=True))
    scale = np.maximum(np.abs(b), rms)
    diff = np.abs(a - b)
    return np.where(scale > 0, diff / np.where(scale > 0, scale, 1.0), np.where(diff > 0, np.inf, 0.0))


def test_get_rms_python_matches_reference_driver():
    # cpp-main.cpp:12-17: DIGITAL_FILTER df(config); df.get_rms()  (500 x dt = 1e-5)
    g = np.load(os.path.join(GOLDEN, "rms_native_s42.npz"))
    f = dfamd.DigitalFilter(seed=int(g["seed"]), device=0)
    f.rms_reset()
    for _ in range(500):
        f.filter(1e-5)
        f.rms_add()
    rows = list(g["sample_rows"])
    for k in FIELDS:
        r = f.rms(k)
        # 500 bit-identical steps, the same per-cell accumulation order and IEEE sqrt(acc / count): the
        # reference's RMS bit for bit (df.cpp:571-582, 615-621)
        bad = np.flatnonzero(r[rows].ravel() != g[f"rms_{k}_rows"].ravel())
        assert bad.size == 0, (k, bad.size, r[rows].ravel()[bad[:1]], g[f"rms_{k}_rows"].ravel()[bad[:1]])
        st = np.array([r.sum(), (r * r).sum(), np.abs(r).max()])
        assert np.allclose(st, g[f"rms_{k}_stats"], rtol=1e-12), k


def test_cpp_driver_get_rms_csv(tmp_path):
    assert os.path.exists(EXE), "examples/cpp-test not built (__graft_entry__.build())"
    run = tmp_path / "run"
    (tmp_path / "files").mkdir()
    run.mkdir()
    out = subprocess.run([EXE, "rms", "42"], cwd=run, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "Finished plotting to file" in out.stdout
    mine = open(tmp_path / "files" / "cpp_vel_fluc_rms.csv").read().splitlines()
    ref = open(os.path.join(GOLDEN, "rms_native_s42_csv_head.txt")).read().splitlines()
    assert mine[0] == ref[0]
    assert len(mine) == 510 * 400 + 1
    for a, b in zip(mine[1:len(ref)], ref[1:]):
        va = np.array([float(x) for x in a.split(",")])
        vb = np.array([float(x) for x in b.split(",")])
        assert np.allclose(va, vb, rtol=2e-6, atol=0), (a, b)


@pytest.mark.parametrize("ordered", [False, True])
def test_cpp_driver_filter_csv_matches_oracle(tmp_path, ordered):
    # ordered: DFConfig::stream_ordered with host_mirror 0 - filter() never waits on the host
    csv = tmp_path / "g.csv"
    out = subprocess.run([EXE, "synth", "64", "96", "2", "10", "17", "3", str(csv)] + (["ordered"] if ordered else []),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.count("Filtering took") == 3
    o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=64, Nz=96, N_min=2, N_max=10, seed=17)
    for _ in range(3):
        o.filter(1e-8)
    ref = tmp_path / "o.csv"
    o.write_csv(str(ref))
    A = np.loadtxt(csv, delimiter=",", skiprows=1)
    B = np.loadtxt(ref, delimiter=",", skiprows=1)
    assert A.shape == B.shape == (64 * 96, 7)
    assert np.array_equal(A[:, :2], B[:, :2])  # coordinates: identical text
    assert float(np.abs(A - B).max()) <= 1e-9 * max(1.0, float(np.abs(B).max()))


def test_cpp_two_objects_share_the_process_stream(tmp_path):
    # df.cpp:334-335: the pcg32 and normal_distribution are function-local statics, so a second
    # DIGITAL_FILTER continues the stream of the first, in call order (DFConfig::shared_stream).
    # The oracle keeps a pointer to its Rng: two oracle filters on one Rng are the reference's statics.
    a_csv, b_csv = tmp_path / "a.csv", tmp_path / "b.csv"
    out = subprocess.run([EXE, "twin", "40", "72", "2", "8", "23", "2", str(a_csv), str(b_csv)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    rng = O.Rng(seed=23)
    oa = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=40, Nz=72, N_min=2, N_max=8, rng=rng)
    ob = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=40, Nz=72, N_min=2, N_max=8, rng=rng)
    for _ in range(2):
        oa.filter(1e-8)
        ob.filter(1e-8)
    for csv, o, name in ((a_csv, oa, "oa.csv"), (b_csv, ob, "ob.csv")):
        ref = tmp_path / name
        o.write_csv(str(ref))
        A = np.loadtxt(csv, delimiter=",", skiprows=1)
        B = np.loadtxt(ref, delimiter=",", skiprows=1)
        assert A.shape == B.shape == (40 * 72, 7)
        assert np.array_equal(A[:, :2], B[:, :2])
        assert float(np.abs(A - B).max()) <= 1e-9 * max(1.0, float(np.abs(B).max())), name
    # the two objects drew different parts of the stream
    A = np.loadtxt(a_csv, delimiter=",", skiprows=1)
    B = np.loadtxt(b_csv, delimiter=",", skiprows=1)
    assert float(np.abs(A[:, 2:] - B[:, 2:]).max()) > 0


def _hip_memcpy_d2h(dst, src_ptr, nbytes):
    """hipMemcpy on the null stream: the handle's streams are non-blocking, so this copy waits for none of
    them - whatever the field holds once the host returns from df_wait is what it reads."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipMemcpy(ctypes.c_void_p(dst.ctypes.data), ctypes.c_void_p(src_ptr), ctypes.c_size_t(nbytes), 2)
    assert rc == 0, rc


@pytest.mark.parametrize("plane", [dict(plane="native"), dict(plane="synthetic", Ny=512, Nz=512, N_min=4, N_max=32)])
@pytest.mark.parametrize("mode", ["table", "packed"])
def test_df_wait_covers_the_call_fields(plane, mode):
    # df_wait waits for the handle's stream only - not the RNG stream / ystream carrying later calls' noise and
    # y-passes - and that is every write a filter() result depends on: after 6 asynchronous calls and one
    # df_wait, a copy that orders after none of the handle's streams reads the oracle's fields
    f = dfamd.DigitalFilter(seed=31, device=0, coeff_mode=mode, **plane)
    o = O.Filter(plane=O.PLANE_NATIVE, seed=31) if plane["plane"] == "native" else O.Filter(
        plane=O.PLANE_SYNTHETIC, Ny=plane["Ny"], Nz=plane["Nz"], N_min=plane["N_min"], N_max=plane["N_max"], seed=31)
    for _ in range(6):
        f.filter(1e-8)
        o.filter(1e-8)
    f.wait()
    for i, k in enumerate(FIELDS):
        ref = o.field(k)
        got = np.empty_like(ref)
        _hip_memcpy_d2h(got, f.device_ptr(k), got.nbytes)
        assert np.array_equal(got, ref), k
    assert f.rng_state() == o.rng.state


def test_variance_invariant_over_time():
    """sum b^2 = 1 and the variance-preserving correlation give
    Var(u') -> R11, Cov(u',v') -> R21, Var(v') -> R22, Var(w') -> R33 per row."""
    f = dfamd.DigitalFilter(plane="synthetic", Ny=64, Nz=1024, N_min=2, N_max=6, seed=3, device=0)
    acc = {k: np.zeros(64) for k in ("uu", "uv", "vv", "ww")}
    n = 0
    for _ in range(60):
        f.filter(1e-5)  # alpha ~ 4e-12: nearly independent samples
        u, v, w = f.field("u"), f.field("v"), f.field("w")
        acc["uu"] += (u * u).mean(axis=1)
        acc["uv"] += (u * v).mean(axis=1)
        acc["vv"] += (v * v).mean(axis=1)
        acc["ww"] += (w * w).mean(axis=1)
        n += 1
    R = {k: f.row(k) for k in ("R11", "R21", "R22", "R33")}
    rows = slice(8, 60)  # rows with R11 well above zero
    for got, want in (("uu", "R11"), ("vv", "R22"), ("ww", "R33")):
        ratio = (acc[got][rows] / n) / R[want][rows]
        assert np.all(np.abs(ratio - 1) < 0.08), (got, ratio.min(), ratio.max())
    cov = acc["uv"][rows] / n
    assert np.all(np.abs(cov - R["R21"][rows]) < 0.1 * np.sqrt(R["R11"][rows] * R["R22"][rows]))


def test_cpp_mirrors_follow_moved_or_reallocated_vectors():
    # u.fluc etc. are the caller's vectors, page-locked by the wrapper; moving, swapping or
    # re-allocating them between filter() calls must not leave a stale or freed registration behind
    out = subprocess.run([EXE, "remirror"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "remirror ok" in out.stdout
