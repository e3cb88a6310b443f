"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's golden vectors.

Bar (SURVEY 8c / BASELINE north_star):
  * pcg32 stream position, polar accept decisions and the cached normal:
    bit-exact (checked through the stream state after every call);
  * fields u', v', w', T', rho': bit-identical to the oracle and to the reference's
    own fixtures (np.array_equal) on every plane kind: synthetic, the reference's grid,
    per-cell half-widths on real grids, z-strips. SURVEY 8c's looser bar
    (|a - b| <= 1e-6 * max(|b|, RMS_row(b)), TOL below) is kept only for the
    fast_log 0/1 noise variants, whose log is not glibc's.
"""
import os

import numpy as np
import pytest

import dfamd
import oracle as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

TOL = 1e-6
FIELDS = ("u", "v", "w", "T", "rho")


def rel_err(a, b):
    rms = np.sqrt((b * b).mean(axis=-1, keepdims=True))
    scale = np.maximum(np.abs(b), rms)
    diff = np.abs(a - b)
    return np.where(scale > 0, diff / np.where(scale > 0, scale, 1.0), np.where(diff > 0, np.inf, 0.0))


def assert_fields(gpu, ref, tol=TOL, what=""):
    worst = {}
    for k in FIELDS:
        a, b = gpu[k], ref[k]
        assert a.shape == b.shape, (k, a.shape, b.shape)
        assert np.isfinite(a).all(), k
        e = float(rel_err(a, b).max())
        worst[k] = e
        assert e <= tol, f"{what} field {k}: rel err {e:.3e} > {tol}"
    return worst


def assert_same(a, b, what=""):
    """Bit-identity with the first differing cell named."""
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    if not np.array_equal(a, b):
        bad = np.argwhere(a != b)
        i = tuple(int(x) for x in bad[0])
        raise AssertionError(f"{what}: {len(bad)} cells differ; first at {i}: {a[i]!r} vs {b[i]!r}")


def assert_stats(a, ref, what=""):
    st3 = np.array([a.sum(), (a * a).sum(), np.abs(a).max()])
    assert np.allclose(st3, ref, rtol=1e-12, atol=1e-300), (what, st3, ref)


def oracle_synth(Ny, Nz, N_min, N_max, seed=None, rng=None):
    return O.Filter(plane=O.PLANE_SYNTHETIC, Ny=Ny, Nz=Nz, N_min=N_min, N_max=N_max, seed=seed, rng=rng)


def gpu_synth(Ny, Nz, N_min, N_max, **kw):
    return dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=N_min, N_max=N_max, device=0, **kw)


# ---------------------------------------------------------------- RNG stream

@pytest.mark.parametrize("spec", [(37, 5, 2, 10), (128, 128, 8, 8), (96, 300, 4, 20)])
def test_rng_stream_state_bitexact(spec):
    o = oracle_synth(*spec, seed=7)
    g = gpu_synth(*spec, seed=7)
    assert g.stream_length() == sum(O.stream_lengths(o))
    assert g.rng_state() == o.rng.state
    for dt in (1e-8, 1e-5, 1e-8):
        o.filter(dt)
        g.filter(dt)
        assert g.rng_state() == o.rng.state


@pytest.mark.parametrize("fast_log", ["2", "1", "0"])
def test_noise_arrays_match_oracle(fast_log):
    # fast_log 2 (default): glibc's own log (df_rng.hpp glibc_log): the normals are the reference's bits;
    # 1: the table-driven log_r2; 0: the device library's log (both within 2 ulp)
    spec = (64, 200, 2, 12)
    o = oracle_synth(*spec, seed=11)
    g = gpu_synth(*spec, seed=11, tuning=dict(fast_log=int(fast_log)))
    o.filter(1e-8)
    g.filter(1e-8)
    diff_ulps = []
    for c in range(3):
        F = o.comp(c)
        ry_o = np.ctypeslib.as_array(F.r_ys, shape=(F.r_ys_size,)).reshape(-1, o.Nz)
        ry_g = g.noise(c, "y")
        assert ry_g.shape == ry_o.shape
        ulp = np.abs(ry_g.view(np.int64) - ry_o.view(np.int64))
        diff_ulps.append(int(ulp.max()))
        assert ulp.max() <= (0 if fast_log == "2" else 2), f"normals differ by {ulp.max()} ulp"
        rz_o = np.ctypeslib.as_array(F.r_zs, shape=(F.r_zs_size,)).reshape(o.Ny, -1)
        rz_g = g.noise(c, "z")
        assert rz_g.shape == rz_o.shape
        assert float(rel_err(rz_g, rz_o).max()) <= 1e-12
        if fast_log == "2":
            assert np.array_equal(rz_g, rz_o)  # pads raw noise, interior y-filtered: the reference's bits
    print("max ulp diff of normals per component:", diff_ulps)


def test_resume_continues_stream_exactly():
    spec = (48, 64, 2, 8)
    a = gpu_synth(*spec, seed=5)
    a.filter(1e-8)
    st = a.rng_state()
    fo = a.field("filt_old_u")
    b = gpu_synth(*spec, resume=st)
    # b ran its own step 0 from st: same stream as a's next call
    a.filter(1e-8)
    assert a.rng_state() == b.rng_state()
    assert fo.shape == (48, 64)


# ------------------------------------------------------- golden (reference) cases

def check_golden_case(name, coeff_mode="packed", rows_per_wave=8):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    Ny, Nz = int(g["Ny"]), int(g["Nz"])
    st = (int(g["start_state"]), int(g["start_saved_flag"]), float(g["start_saved"]))
    f = gpu_synth(Ny, Nz, int(g["N_min"]), int(g["N_max"]), resume=st, coeff_mode=coeff_mode,
                  rows_per_wave=rows_per_wave)
    rows = list(g["sample_rows"])
    full = set(int(x) for x in g["full_steps"])
    dts = [float(g["dt"])] * int(g["nsteps"]) + [float(g["dt2"])] * int(g["nsteps2"])
    for s, dt in enumerate([None] + dts):
        if dt is not None:
            f.filter(dt)
        got = f.fields()
        for k in FIELDS:
            a = got[k]
            assert_same(a[rows], g[f"s{s}_{k}_rows"], f"{name} step {s} {k} rows")
            assert_stats(a, g[f"s{s}_{k}_stats"], (name, s, k))
            if s in full:
                assert_same(a, g[f"s{s}_{k}"], f"{name} step {s} {k}")
            if f"s{s}_{k}_sha256" in g:  # the whole field bit for bit against the reference's own output
                assert field_sha256(a) == str(g[f"s{s}_{k}_sha256"]), (name, s, k)
    return f


def field_sha256(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["c1_s42", "ramp256_s1234", "ragged_s7"])
def test_golden_synthetic(name):
    check_golden_case(name)


@pytest.mark.parametrize("mode", ["packed", "table"])
def test_golden_c2_bitexact_vs_reference(mode):
    # c2 (BASELINE configs[1], 512 x 512, N 4-32) against the reference's own output (tests/golden/c2_s42.npz,
    # oracle/gen_golden.py: df.cpp compiled here): every whole field at step 0 and after two calls, by sha256
    check_golden_case("c2_s42", coeff_mode=mode, rows_per_wave=0)


@pytest.mark.parametrize("mode,tuning", [("packed", {}), ("packed", dict(rows_per_wave=1, yunroll=8, ycoop=0)),
                                         ("packed", dict(zsplit=1)), ("packed", dict(ycoop=7, ycoop_order=1)),
                                         ("table", dict(ylds=0, rows_per_wave=4)), ("table", dict(gen_dense=2)),
                                         ("table", dict(ylds=3, yt_rows=2))])
def test_golden_native_grid(mode, tuning):
    # the reference's own grid (N_y up to 212): default shapes and the deep y-pass pipeline
    g = np.load(os.path.join(GOLDEN, "native_s42.npz"))
    f = dfamd.DigitalFilter(seed=42, device=0, coeff_mode=mode)
    for k, v in tuning.items():
        f.set_tuning(k, v)
    assert (f.Ny, f.Nz) == (510, 400)
    rows = list(g["sample_rows"])
    for s in range(int(g["nsteps"]) + 1):
        if s:
            f.filter(float(g["dt"]))
        got = f.fields()
        for k in FIELDS:
            assert_same(got[k][rows], g[f"s{s}_{k}_rows"], f"native step {s} {k} rows")
            assert_stats(got[k], g[f"s{s}_{k}_stats"], (s, k))


@pytest.mark.parametrize("mode,tuning", [("packed", {}), ("packed", dict(ycoop=0)), ("packed", dict(ycoop_order=1)),
                                         ("packed", dict(ycoop_order=8)), ("packed", dict(ycoop_split=96)),
                                         ("packed", dict(ycoop_split=1, ycoop_order=0)), ("packed", dict(ycoop_split=0)),
                                         ("packed", dict(ycoop_split4=160)), ("packed", dict(ycoop_split4=1, ycoop_split=0)),
                                         ("table", {}), ("table", dict(rows_per_wave=1)),
                                         ("table", dict(ylds=1)), ("table", dict(ylds=2, rows_per_wave=2)),
                                         ("table", dict(ylds=3, rows_per_wave=4)), ("table", dict(ylds=3)),
                                         ("table", dict(ylds=3, yt_rows=1)), ("table", dict(ylds=3, yt_rows=2)),
                                         ("table", dict(ylds=3, yt_rows=1, yt_pd=4)), ("table", dict(ylds=3, yt_rows=2, yt_chunk=8)),
                                         ("table", dict(ylds=3, yt_rows=1, yt_chunk=24)),
                                         ("table", dict(ylds=0))])
def test_native_grid_bitexact_vs_oracle(mode, tuning):
    # the whole 510 x 400 plane of the reference's grid against the live oracle, bit for bit: the row-pair
    # y-pass (packed default, its 16-column last strip folded 8 noise rows per load) and the table path
    o = O.Filter(plane=O.PLANE_NATIVE, seed=42)
    g = dfamd.DigitalFilter(seed=42, device=0, coeff_mode=mode)
    for k, v in tuning.items():
        g.set_tuning(k, v)
    for dt in (None, 1e-8, 1e-5):
        if dt is not None:
            o.filter(dt)
            g.filter(dt)
        gf, of = g.fields(), o.fields()
        for k in FIELDS:
            assert np.array_equal(gf[k], of[k]), (dt, k, float(np.abs(gf[k] - of[k]).max()))
        assert g.rng_state() == o.rng.state


# -------------------------------------------------------------- live oracle

@pytest.mark.parametrize("spec", [(128, 128, 8, 8), (37, 5, 2, 10), (2, 1, 2, 2), (70, 129, 2, 6), (24, 257, 4, 12)])
def test_fields_vs_oracle(spec):
    o = oracle_synth(*spec, seed=3)
    g = gpu_synth(*spec, seed=3)
    gf, of = g.fields(), o.fields()
    for k in FIELDS:
        assert_same(gf[k], of[k], f"step0 {k}")
    for dt in (1e-8, 1e-8, 1e-5):
        o.filter(dt)
        g.filter(dt)
        gf, of = g.fields(), o.fields()
        for k in FIELDS:
            assert_same(gf[k], of[k], f"dt={dt} {k}")
    for c in range(3):
        assert np.array_equal(g.field(f"filt_old_{'uvw'[c]}").shape, (o.Ny, o.Nz))


@pytest.mark.parametrize("mode", ["packed", "table"])
@pytest.mark.parametrize("spec", [(128, 128, 8, 8), (37, 5, 2, 10), (70, 129, 2, 6), (96, 300, 4, 20)])
def test_fields_bitexact_vs_oracle(spec, mode):
    # with glibc's log in K3 (the default) the noise is the reference's bit for bit, and the sweeps and
    # the epilogue round every product and sum as df.cpp does: every field equals the oracle's exactly
    o = oracle_synth(*spec, seed=3)
    g = gpu_synth(*spec, seed=3, coeff_mode=mode)
    for dt in (None, 1e-8, 1e-8, 1e-5):
        if dt is not None:
            o.filter(dt)
            g.filter(dt)
        gf, of = g.fields(), o.fields()
        for k in FIELDS:
            assert np.array_equal(gf[k], of[k]), (dt, k, float(np.abs(gf[k] - of[k]).max()))
        assert g.rng_state() == o.rng.state


def test_golden_c1_bitexact():
    # the reference's own output (df.cpp built here, tests/golden/c1_s42.npz full steps): bit for bit
    g = np.load(os.path.join(GOLDEN, "c1_s42.npz"))
    st = (int(g["start_state"]), int(g["start_saved_flag"]), float(g["start_saved"]))
    f = gpu_synth(int(g["Ny"]), int(g["Nz"]), int(g["N_min"]), int(g["N_max"]), resume=st)
    full = set(int(x) for x in g["full_steps"])
    dts = [float(g["dt"])] * int(g["nsteps"]) + [float(g["dt2"])] * int(g["nsteps2"])
    checked = 0
    for s, dt in enumerate([None] + dts):
        if dt is not None:
            f.filter(dt)
        if s in full:
            got = f.fields()
            for k in FIELDS:
                assert np.array_equal(got[k], g[f"s{s}_{k}"]), (s, k)
            checked += 1
    assert checked >= 1


def test_c2_512_variable_halfwidth_vs_oracle():
    spec = (512, 512, 4, 32)
    o = oracle_synth(*spec, seed=1234)
    g = gpu_synth(*spec, seed=1234)
    for dt in (1e-8, 1e-8):
        o.filter(dt)
        g.filter(dt)
    assert g.rng_state() == o.rng.state
    gf, of = g.fields(), o.fields()
    for k in FIELDS:
        assert_same(gf[k], of[k], f"c2 {k}")


# ------------------------------------------------------- variants are identical

def run_variant(spec, steps=2, **kw):
    g = gpu_synth(*spec, seed=99, **kw)
    for _ in range(steps):
        g.filter(1e-8)
    return g.fields()


def test_table_mode_bitexact_with_packed():
    spec = (200, 300, 4, 24)
    a = run_variant(spec, coeff_mode="packed")
    b = run_variant(spec, coeff_mode="table")
    for k in FIELDS:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("rpw", [1, 2, 8])
def test_rows_per_wave_bitexact(rpw):
    spec = (131, 260, 2, 16)
    a = run_variant(spec, rows_per_wave=4)
    b = run_variant(spec, rows_per_wave=rpw)
    for k in FIELDS:
        assert np.array_equal(a[k], b[k]), (rpw, k)


@pytest.mark.parametrize("mode", ["packed", "table"])
def test_runtime_tuning_is_bitexact(mode):
    # df_set_tuning flips launch shapes between calls; fields must not move by one bit
    spec = (131, 260, 2, 16)
    a = gpu_synth(*spec, seed=5, coeff_mode=mode)
    b = gpu_synth(*spec, seed=5, coeff_mode=mode)
    settings = [dict(ypass_ahead=1), dict(rows_per_wave=1, yunroll=4), dict(rows_per_wave=8),
                dict(rows_per_wave=2, yunroll=2, nt_stores=1), dict(nt_stores=0), dict(rows_per_wave=1, yunroll=8),
                dict(rows_per_wave=4, yunroll=8), dict(gen_split=1), dict(gen_split=4), dict(gen_split=16),
                dict(ywin_T=1024, ywin_W=64, zwin_T=2048, zwin_W=256), dict(ywin_T=0, zwin_T=4096, zwin_W=0),
                dict(gen_split=2), dict(zsplit=1), dict(zsplit=0), dict(ycoop=7), dict(ycoop=7, ycoop_order=1), dict(ycoop=7, ycoop_order=4), dict(ycoop_split=8), dict(ycoop_order=0), dict(ycoop_split=12), dict(ycoop_split4=10), dict(ycoop_split=0), dict(ycoop_split4=0),
                dict(ycoop=0, yunroll=2), dict(rows_per_wave=2), dict(rows_per_wave=1), dict(rows_per_wave=8),
                dict(fuse_plan=0, gen_split=1, gen_dense=2),
                dict(fuse_plan=0), dict(fuse_plan=1, gen_split=4), dict(fuse_plan=0, gen_split=2), dict(fuse_plan=1, gen_split=1),
                dict(gen_dense=0), dict(handoff_batch=1), dict(handoff_batch=2), dict(handoff_batch=4),
                dict(ylds=1, rows_per_wave=1), dict(ylds=1, rows_per_wave=2), dict(ylds=1, rows_per_wave=4),
                dict(ylds=1, rows_per_wave=8), dict(ylds=0), dict(ypass_ahead=0), dict(ypass_ahead=1)]
    if mode == "table":  # 64-column tiles (ypass_t64_kernel), every row count, then back
        settings += [dict(ylds=3, yt_rows=1), dict(yt_rows=2), dict(yt_chunk=8), dict(yt_rows=1, yt_pd=4), dict(yt_pd=2),
                     dict(yt_chunk=24),
                     dict(yt_rows=2, yt_chunk=16), dict(ylds=2), dict(ylds=0)]
    for kw in settings:
        for k, v in kw.items():
            b.set_tuning(k, v)
        a.filter(1e-8)
        b.filter(1e-8)
        for k in FIELDS:
            assert np.array_equal(a.field(k), b.field(k)), (kw, k)
        assert a.rng_state() == b.rng_state(), kw
    with pytest.raises(dfamd.DFError, match="unknown tuning"):
        b.set_tuning("warp_size", 32)
    with pytest.raises(dfamd.DFError, match="rows_per_wave"):
        b.set_tuning("rows_per_wave", 3)
    with pytest.raises(dfamd.DFError, match="power of two"):
        b.set_tuning("zwin_T", 3000)
    with pytest.raises(dfamd.DFError, match="handoff_batch"):
        b.set_tuning("handoff_batch", 3)


@pytest.mark.parametrize("hb", ["1", "2", "4"])
def test_handoff_batch_mid_epoch_state_changes(hb):
    # epochs of hb calls over 2*hb noise sets: a stream state set mid-epoch, the stage API and filter calls
    # interleaved, checked against the oracle after every step
    spec = (48, 96, 2, 10)
    o = oracle_synth(*spec, seed=13)
    g = gpu_synth(*spec, seed=13, tuning=dict(handoff_batch=int(hb)))
    # a loaded state drops the handle to one generation per epoch; 16 calls later it batches again
    # (kHbRestoreCalls): loads at calls 2, 3 and 22 cover the drop, the return and a drop after it
    for i in range(26):
        o.filter(1e-8)
        g.filter(1e-8)
        if i in (2, 3, 22):  # mid-epoch: restart the pipeline from the oracle's current state
            st = o.rng.state
            g.set_rng_state(*st)
        assert g.rng_state() == o.rng.state, i
        for k in FIELDS:
            assert np.array_equal(g.field(k), o.field(k)), (i, k)


@pytest.mark.parametrize("spec", [(131, 700, 2, 16), (57, 1100, 3, 90), (37, 129, 2, 10), (40, 133, 2, 8)])
def test_dense_fast_chunks_match_oracle(spec):
    # the run generation's fast chunks (host-built destinations, ChunkDest) forced on small planes: odd and even
    # widths (row wraps inside a chunk, odd wrap points), both parities of the carried normal
    o = oracle_synth(*spec, seed=29)
    g = gpu_synth(*spec, seed=29, coeff_mode="table", tuning=dict(gen_split=1, fuse_plan=0, gen_dense=2))
    flags = set()
    for i in range(5):
        o.filter(1e-8)
        g.filter(1e-8)
        st = g.rng_state()
        flags.add(st[1])
        assert st == o.rng.state, i
        for k in FIELDS:
            assert np.array_equal(g.field(k), o.field(k)), (i, k)
    print("saved flags seen:", sorted(flags))


def test_random_planes_bitexact_vs_oracle():
    # seeded random plane shapes and half-width ranges, both coefficient modes, table mode also through the
    # dense generation (fast chunks) and the LDS-staged y-pass (ylds), the packed mode through the row-pair y-pass
    # with its dispatch orders:
    # every field bit for bit against the oracle after step 0 and two calls
    rs = np.random.RandomState(2024)
    for case in range(10):
        Ny, Nz = int(rs.randint(3, 200)), int(rs.randint(2, 700))
        lo = 2 * int(rs.randint(1, 6))
        hi = lo + 2 * int(rs.randint(0, 12))
        seed = int(rs.randint(1, 1 << 30))
        o = oracle_synth(Ny, Nz, lo, hi, seed=seed)
        hs = {"packed": gpu_synth(Ny, Nz, lo, hi, seed=seed, coeff_mode="packed"),
              "table": gpu_synth(Ny, Nz, lo, hi, seed=seed, coeff_mode="table"),
              "dense": gpu_synth(Ny, Nz, lo, hi, seed=seed, coeff_mode="table"),
              "coop2": gpu_synth(Ny, Nz, lo, hi, seed=seed, coeff_mode="packed"),
              "tlds": gpu_synth(Ny, Nz, lo, hi, seed=seed, coeff_mode="table")}
        hs["tlds"].set_tuning("ylds", 2)
        hs["tlds"].set_tuning("rows_per_wave", int(rs.choice([1, 2, 4])))
        for k, v in (("gen_split", 1), ("fuse_plan", 0), ("gen_dense", 2)):
            hs["dense"].set_tuning(k, v)
        hs["coop2"].set_tuning("ycoop", 7)
        hs["coop2"].set_tuning("ycoop_order", int(rs.choice([0, 1, 4])))
        for step in range(3):
            if step:
                o.filter(1e-8)
                for g in hs.values():
                    g.filter(1e-8)
            of = o.fields()
            for name, g in hs.items():
                assert g.rng_state() == o.rng.state, (case, name, step)
                gf = g.fields()
                for k in FIELDS:
                    assert np.array_equal(gf[k], of[k]), (case, (Ny, Nz, lo, hi), name, step, k)


@pytest.mark.parametrize("spec", [(131, 700, 2, 16), (57, 1100, 3, 90)])
def test_table_lds_staging_is_bitexact(spec):
    # 6 and 9 strips: some blocks hold 4 strips of one row (noise staged in LDS), others
    # straddle two rows (global path); zstage=0 forces the global path everywhere
    a = gpu_synth(*spec, seed=8, coeff_mode="table")
    b = gpu_synth(*spec, seed=8, coeff_mode="table")
    p = gpu_synth(*spec, seed=8, coeff_mode="packed")
    b.set_tuning("zstage", 0)
    for _ in range(2):
        for f in (a, b, p):
            f.filter(1e-8)
        for k in FIELDS:
            assert np.array_equal(a.field(k), b.field(k)), k
            assert np.array_equal(a.field(k), p.field(k)), k


@pytest.mark.parametrize("spec", [(131, 700, 2, 16), (57, 1100, 3, 90), (64, 130, 2, 8), (33, 257, 2, 12)])
def test_table_zstage_copies_are_bitexact(spec):
    # the staging copies of the table z-pass (0 none; 1 and 2 both the 16-B copy with loads first):
    # full and partial groups of 4 strips (6, 9, 2 and 3 strips), odd and even Nz, against packed
    hs = [gpu_synth(*spec, seed=8, coeff_mode="table") for _ in range(3)]
    p = gpu_synth(*spec, seed=8, coeff_mode="packed")
    for level, h in enumerate(hs):
        h.set_tuning("zstage", level)
    for _ in range(3):
        for f in hs + [p]:
            f.filter(1e-8)
        for k in FIELDS:
            for h in hs:
                assert np.array_equal(h.field(k), p.field(k)), k
    assert all(h.rng_state() == p.rng_state() for h in hs)


def test_gather_field_device_handoff():
    import torch
    f = gpu_synth(40, 33, 2, 6, seed=3)
    f.filter(1e-8)
    n = f.Ny * f.Nz_loc
    u = torch.from_numpy(f.field("u").ravel()).cuda()
    dst = torch.zeros(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    f.gather("u", dst.data_ptr(), n, n)  # identity copy, beta = 0
    f.sync()
    assert torch.equal(dst, u)
    perm = torch.randperm(n, device="cuda")
    base = torch.arange(n, dtype=torch.float64, device="cuda")
    dst2 = base.clone()
    torch.cuda.synchronize()
    f.gather("u", dst2.data_ptr(), n, n, plane_cell=perm.data_ptr(), beta=1.0)  # dst += u[perm]
    f.sync()
    assert torch.equal(dst2, base + u[perm])
    bad = torch.full((4,), n + 5, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    f.gather("u", dst.data_ptr(), 4, n, plane_cell=bad.data_ptr())
    with pytest.raises(dfamd.DFError, match="out-of-range"):
        f.sync()
    f.sync()  # reported once
    with pytest.raises(dfamd.DFError, match="dst_len"):
        f.gather("u", dst.data_ptr(), n + 1, n, plane_cell=perm.data_ptr())


def test_stage_api_matches_filter():
    spec = (96, 150, 2, 10)
    a = gpu_synth(*spec, seed=21)
    b = gpu_synth(*spec, seed=21)
    a.filter(1e-8)
    # df.cpp:449-461 spelled out through the public stage functions
    b.generate_white_noise()
    for c in range(3):
        b.filtering_sweeps(c)
        b.correlate_fields(c, 1e-8)
    b.apply_RST_scaling()
    b.get_rho_T_fluc()
    fa, fb = a.fields(), b.fields()
    for k in FIELDS:
        assert np.array_equal(fa[k], fb[k]), k
    assert a.rng_state() == b.rng_state()


@pytest.mark.parametrize("world,Nz,mode", [(2, 256, "packed"), (3, 256, "packed"), (2, 1100, "table"),
                                            (3, 1700, "table")])
def test_z_strips_in_process_match_single(world, Nz, mode):
    # table cases: 4-5 strips per rank, so some blocks stage their row's noise (halo from
    # the neighbour included) in LDS and others straddle rows
    spec = dict(plane="synthetic", Ny=100, Nz=Nz, N_min=4, N_max=16, seed=8, device=0, coeff_mode=mode)
    whole = dfamd.DigitalFilter(**spec)
    strips = dfamd.create_group(world, **spec)
    for _ in range(2):
        whole.filter(1e-8)
        dfamd.filter_group(strips, 1e-8)
    for k in FIELDS:
        cat = np.concatenate([s.field(k) for s in strips], axis=1)
        assert np.array_equal(cat, whole.field(k)), k
    assert all(s.rng_state() == whole.rng_state() for s in strips)


def test_rccl_single_rank_matches_plain():
    # The RCCL calls of the z-strip path (ncclCommInitRank, ncclCommSplit, the grouped in-place
    # ncclAllGather of block counts, wave counts and accept masks on the RNG stream) run here with a
    # communicator of one rank; results must equal the plain single-GPU handle bit for bit.
    spec = dict(plane="synthetic", Ny=96, Nz=300, N_min=4, N_max=16, seed=5, device=0)
    plain = dfamd.DigitalFilter(**spec)
    rc = dfamd.DigitalFilter(rank=0, world=1, comm_id=dfamd.comm_unique_id(), **spec)
    for dt in (1e-8, 1e-8, 1e-5):
        plain.filter(dt)
        rc.filter(dt)
        for k in FIELDS:
            assert np.array_equal(rc.field(k), plain.field(k)), k
        assert rc.rng_state() == plain.rng_state()
    rc.close()
    plain.close()


def test_rccl_halo_send_recv_loopback():
    # The z-strip halo exchange (grouped ncclSend/ncclRecv of the packed edge columns, all three
    # components) on one GPU: a one-rank communicator sends both plane edges to itself each call and
    # the device compares what arrived with what was sent. Fields stay bit-identical to the plain
    # handle (the received columns are not unpacked); a corrupted element must be reported.
    spec = dict(plane="synthetic", Ny=96, Nz=300, N_min=4, N_max=16, seed=9, device=0)
    plain = dfamd.DigitalFilter(**spec)
    rc = dfamd.DigitalFilter(rank=0, world=1, comm_id=dfamd.comm_unique_id(), **spec)
    with pytest.raises(dfamd.DFError):
        plain.set_tuning("halo_loopback", 1)  # needs a communicator
    rc.set_tuning("halo_loopback", 1)
    for dt in (1e-8, 1e-8):
        plain.filter(dt)
        rc.filter(dt)
    rc.sync()
    for k in FIELDS:
        assert np.array_equal(rc.field(k), plain.field(k)), k
    assert rc.rng_state() == plain.rng_state()
    rc.set_tuning("halo_loopback", 2)  # one received value perturbed: the check must see it
    rc.filter(1e-8)
    with pytest.raises(dfamd.DFError, match="loopback"):
        rc.sync()
    rc.close()
    plain.close()


def test_set_rng_state_discards_prefetched_noise():
    # The next call's noise is generated ahead of time on a second stream; moving the
    # stream must regenerate it (df.cpp:334-335 semantics: draws follow the state).
    spec = (40, 70, 2, 8)
    a = gpu_synth(*spec, seed=1)
    a.filter(1e-8)
    other = gpu_synth(*spec, seed=2)
    st = other.rng_state()
    a.set_rng_state(*st)
    a.generate_white_noise()
    c = gpu_synth(*spec, resume=st)  # its step 0 drew from st
    for comp in range(3):
        assert np.array_equal(a.noise(comp, "y"), c.noise(comp, "y"))
    assert a.rng_state() == c.rng_state()
    # and a no-op reset changes nothing
    x = gpu_synth(*spec, seed=9)
    y = gpu_synth(*spec, seed=9)
    x.filter(1e-8)
    y.filter(1e-8)
    y.set_rng_state(*y.rng_state())
    x.filter(1e-8)
    y.filter(1e-8)
    for k in FIELDS:
        assert np.array_equal(x.field(k), y.field(k))


# ---------------------------------------------------------------- grid planes

def _grid_case(name="grid_s3"):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


@pytest.mark.parametrize("mode,rpw,tuning", [("packed", 0, {}), ("packed", 1, {}), ("packed", 8, {}),
                                             ("packed", 0, dict(ycoop=7)), ("table", 0, {}), ("table", 2, {})])
def test_golden_grid_plane_per_cell_halfwidths(mode, rpw, tuning):
    """Per-cell N (the reference's calculate_filter_properties on a real grid) vs the
    reference's own fields (tests/golden/grid_s3, gen_golden.grid_fixture)."""
    g = _grid_case()
    st = (int(g["start_state"]), int(g["start_saved_flag"]), float(g["start_saved"]))
    f = dfamd.DigitalFilter(plane="grid", grid_y=g["grid_y"], grid_z=g["grid_z"], device=0, resume=st,
                            coeff_mode=mode, rows_per_wave=rpw)
    for k, v in tuning.items():
        f.set_tuning(k, v)
    assert f.plane_info() == (2, True)
    o = O.Filter(plane=O.PLANE_GRID, Ny=int(g["Ny_in"]), Nz=int(g["Nz_in"]), grid_y=g["grid_y"],
                 grid_z=g["grid_z"], rng=O.Rng(state=st[0], saved_flag=st[1], saved=st[2]))
    assert f.rng_state() == o.rng.state
    full = set(int(x) for x in g["full_steps"])
    for s in range(int(g["nsteps"]) + 1):
        if s:
            f.filter(float(g["dt"]))
            o.filter(float(g["dt"]))
            assert f.rng_state() == o.rng.state
        for k in FIELDS:
            a = f.field(k)
            assert_stats(a, g[f"s{s}_{k}_stats"], (s, k))
            if s in full:  # the reference's own fields on its per-cell N: bit for bit
                assert_same(a, g[f"s{s}_{k}"], f"grid_s3 step {s} {k}")
            assert_same(a, o.field(k), f"grid_s3 vs oracle step {s} {k}")


@pytest.mark.parametrize("mode", ["packed", "table"])
def test_grid_plane_vs_oracle_three_strips(mode):
    # another grid: 3 column strips (Nz = 300), steeper spacing, other phase and seed
    gy, gz = O.warped_grid(40, 300, dz0=3.0e-5, wave=0.2, seed_phase=1.0)
    f = dfamd.DigitalFilter(plane="grid", grid_y=gy, grid_z=gz, device=0, seed=17, coeff_mode=mode)
    o = O.Filter(plane=O.PLANE_GRID, Ny=40, Nz=300, grid_y=gy, grid_z=gz, seed=17)
    assert f.plane_info()[1]
    for dt in (None, 1e-8, 2e-8):
        if dt is not None:
            f.filter(dt)
            o.filter(dt)
        assert f.rng_state() == o.rng.state
        for k in FIELDS:
            assert_same(f.field(k), o.field(k), f"grid 3 strips dt={dt} {k}")


def test_grid_plane_table_equals_packed_and_strips_equal_whole():
    g = _grid_case()
    kw = dict(plane="grid", grid_y=g["grid_y"], grid_z=g["grid_z"], device=0, seed=8)
    a = dfamd.DigitalFilter(coeff_mode="packed", **kw)
    b = dfamd.DigitalFilter(coeff_mode="table", **kw)
    strips = dfamd.create_group(2, **kw)
    a.filter(1e-8)
    b.filter(1e-8)
    dfamd.filter_group(strips, 1e-8)
    for k in FIELDS:
        assert np.array_equal(a.field(k), b.field(k)), k
        assert np.array_equal(np.concatenate([s.field(k) for s in strips], axis=1), a.field(k)), k


def test_checkpoint_restore_continues_bitexact():
    """SURVEY 5 checkpoint/resume: stream state + filt_old x3 restored on another handle of the
    same plane (itself at a different point of a different stream) continue the run exactly."""
    spec = (96, 140, 2, 12)
    a = gpu_synth(*spec, seed=5)
    a.filter(1e-8)
    ck = a.checkpoint()
    for _ in range(2):
        a.filter(2e-8)
    b = gpu_synth(*spec, seed=99)
    b.filter(1e-5)
    b.restore(ck)
    for _ in range(2):
        b.filter(2e-8)
    assert b.rng_state() == a.rng_state()
    for k in FIELDS + ("filt_old_u", "filt_old_v", "filt_old_w"):
        assert np.array_equal(a.field(k), b.field(k)), k
    with pytest.raises(dfamd.DFError, match="need"):
        b.set_field("filt_old_u", np.zeros(5))


def test_alloc_registry_tracks_live_handles():
    """The process-wide registry holds every live device range of every handle: a range inside a live
    handle's buffer is refused (DF_EHIP, both ranges named), and destroying the handle releases all
    of its ranges (an allocation aliasing another handle's buffer fails loudly)."""
    import ctypes as C
    L = dfamd.lib()
    L.df_alloc_registry.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    L.df_alloc_registry_count.restype = C.c_longlong
    L.df_device_field.restype = C.c_void_p
    n0 = L.df_alloc_registry_count()
    a = gpu_synth(96, 140, 2, 12, seed=5)
    na = L.df_alloc_registry_count()
    assert na > n0
    b = gpu_synth(96, 140, 2, 12, seed=6, coeff_mode="table")
    assert L.df_alloc_registry_count() > na
    p = L.df_device_field(a._h, 3)  # a's T' buffer
    assert L.df_alloc_registry(p + 64, 64, 1) == -3
    assert "overlaps the live range" in L.df_last_error().decode()
    b.close()
    assert L.df_alloc_registry_count() == na
    a.close()
    assert L.df_alloc_registry_count() == n0


# ---------------------------------------------------------------- randomized sweep of shapes

def _random_cases(n=10, seed=20261015):
    rng = np.random.default_rng(seed)
    cases = []
    for i in range(n):
        kind = "grid" if i % 3 == 2 else "synthetic"
        Ny = int(rng.integers(8, 90))
        Nz = int(rng.integers(1, 300))
        lo = int(rng.integers(1, 6)) * 2
        hi = lo + int(rng.integers(0, 12)) * 2
        mode = "table" if rng.random() < 0.4 else "packed"
        rpw = int(rng.choice([0, 1, 2, 4, 8]))
        world = int(rng.choice([1, 1, 2, 3])) if Nz >= 3 * (hi + 1) else 1
        cases.append(dict(kind=kind, Ny=Ny, Nz=Nz, lo=lo, hi=hi, mode=mode, rpw=rpw, world=world,
                          seed=int(rng.integers(0, 2**31)), phase=float(rng.random() * 6)))
    return cases


@pytest.mark.parametrize("case", _random_cases(), ids=lambda c: "{kind}-{Ny}x{Nz}-N{lo}-{hi}-{mode}-r{rpw}-w{world}".format(**c))
def test_random_planes_vs_oracle(case):
    c = case
    if c["kind"] == "grid":
        Ny, Nz = max(c["Ny"], 20), max(c["Nz"], 4)
        gy, gz = O.warped_grid(Ny, Nz, dz0=3.0e-5, wave=0.15, seed_phase=c["phase"])
        kw = dict(plane="grid", grid_y=gy, grid_z=gz)
        o = O.Filter(plane=O.PLANE_GRID, Ny=Ny, Nz=Nz, grid_y=gy, grid_z=gz, seed=c["seed"])
    else:
        kw = dict(plane="synthetic", Ny=c["Ny"], Nz=c["Nz"], N_min=c["lo"], N_max=c["hi"])
        o = oracle_synth(c["Ny"], c["Nz"], c["lo"], c["hi"], seed=c["seed"])
    kw.update(device=0, seed=c["seed"], coeff_mode=c["mode"], rows_per_wave=c["rpw"])
    try:
        hs = dfamd.create_group(c["world"], **kw) if c["world"] > 1 else [dfamd.DigitalFilter(**kw)]
    except dfamd.DFError as e:  # a z-strip narrower than the z half-width is refused by design
        assert "narrower" in str(e)
        return
    for dt in (None, 1e-8, 3e-8):
        if dt is not None:
            if len(hs) > 1:
                dfamd.filter_group(hs, dt)
            else:
                hs[0].filter(dt)
            o.filter(dt)
        assert all(h.rng_state() == o.rng.state for h in hs)
        for k in FIELDS:
            got = np.concatenate([h.field(k) for h in hs], axis=1)
            assert_same(got, o.field(k), f"dt={dt} {k}")


def test_handles_driven_from_two_host_threads():
    # No hidden process-wide state in the library (the reference's RNG is a process-wide static,
    # df.cpp:334-335; here each handle owns its stream): two handles filtered concurrently from two
    # host threads (ctypes drops the GIL in each call) give exactly the single-threaded results.
    import threading

    specs = [dict(plane="synthetic", Ny=300, Nz=260, N_min=2, N_max=24, seed=s, device=0) for s in (31, 32)]
    ref = []
    for sp in specs:
        f = dfamd.DigitalFilter(**sp)
        for _ in range(5):
            f.filter(1e-8)
        ref.append({k: f.field(k) for k in FIELDS})
        f.close()
    hs = [dfamd.DigitalFilter(**sp) for sp in specs]
    errs = []

    def run(f):
        try:
            for _ in range(5):
                f.filter(1e-8)
            f.sync()
        except Exception as e:  # surfaced below
            errs.append(e)

    ts = [threading.Thread(target=run, args=(f,)) for f in hs]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs, errs
    for f, r in zip(hs, ref):
        for k in FIELDS:
            assert np.array_equal(f.field(k), r[k]), k
        f.close()


def test_sampled_profiling_counts_and_phases():
    # df_set_profiling(h, n): phase events on every n-th call only (bench.py --profile-every)
    f = gpu_synth(64, 200, 2, 12, seed=3)
    a = gpu_synth(64, 200, 2, 12, seed=3)
    f.set_profiling(True, every=4)
    for _ in range(12):
        f.filter(1e-8)
        a.filter(1e-8)
    p = f.profile()
    assert p["calls"] == 3
    assert p["ypass_ms"] > 0 and p["zpass_ms"] > 0 and p["total_ms"] >= p["zpass_ms"]
    f.set_profiling(True)
    for _ in range(5):
        f.filter(1e-8)
        a.filter(1e-8)
    assert f.profile()["calls"] == 5
    f.set_profiling(False)
    for k in FIELDS:  # events never change a result
        assert np.array_equal(f.field(k), a.field(k)), k
