"""Y-pass ahead (round 5, df_handle::yahead): each epoch's y-passes run on a stream of their own as soon as its
noise is generated, calls before the call that consumes them; that call waits for them and runs only the halo
and the z-pass. The y-pass reads nothing but its generation's r_ys and writes nothing but that set's r_zs
interior (df.cpp:359-383), so every field, stream state and noise array must equal the serial form and the
oracle bit for bit - with every hand-off batch, both coefficient modes, the noise forms, strip groups (halo and
ghost columns), the stage API in between, the ahead form switched on and off between calls and a stream state
loaded mid-run."""
import numpy as np
import pytest

import dfamd
import oracle as O

pytestmark = pytest.mark.gpu
FIELDS = ("u", "v", "w", "T", "rho")
AHEAD = dict(ypass_ahead=1)


def synth(spec, seed, mode, tuning=None):
    Ny, Nz, lo, hi = spec
    return dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=seed, device=0,
                               coeff_mode=mode, tuning=tuning)


def same(a, b, what):
    assert a.rng_state() == b.rng_state(), what
    for k in FIELDS:
        x, y = a.field(k), b.field(k)
        if not np.array_equal(x, y):
            bad = np.argwhere(x != y)
            raise AssertionError(f"{what} {k}: {len(bad)} cells differ, first {tuple(bad[0])}")


@pytest.mark.parametrize("mode", ["packed", "table"])
@pytest.mark.parametrize("hb", [1, 2, 4])
def test_ahead_matches_oracle(mode, hb):
    spec = (64, 200, 2, 12)
    o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=64, Nz=200, N_min=2, N_max=12, seed=13)
    g = synth(spec, 13, mode, dict(AHEAD, handoff_batch=hb))
    assert g.get_tuning("ypass_ahead") == 1
    for i, dt in enumerate((1e-8, 1e-8, 1e-5, 1e-8, 1e-8, 1e-8, 1e-8, 1e-8, 1e-8)):
        o.filter(dt)
        g.filter(dt)
        assert g.rng_state() == o.rng.state, i
        for k in FIELDS:
            assert np.array_equal(g.field(k), o.field(k)), (i, k)
    for c in range(3):  # pads raw, interior y-filtered: the reference's r_zs
        F = o.comp(c)
        rz = np.ctypeslib.as_array(F.r_zs, shape=(F.r_zs_size,)).reshape(o.Ny, -1)
        assert np.array_equal(g.noise(c, "z"), rz), c


@pytest.mark.parametrize("mode,tuning", [("packed", {}), ("table", {}), ("table", dict(gen_dense=2, gen_split=1, fuse_plan=0)),
                                         ("table", dict(ylds=3)), ("packed", dict(ycoop=7))])
def test_ahead_toggled_against_serial(mode, tuning):
    spec = (131, 260, 2, 16)
    a = synth(spec, 5, mode, dict(tuning, ypass_ahead=0))
    b = synth(spec, 5, mode, dict(tuning, ypass_ahead=1))
    for i, on in enumerate((1, 1, 0, 1, 1, 1, 0, 0, 1, 1, 1, 1)):
        b.set_tuning("ypass_ahead", on)
        a.filter(1e-8)
        b.filter(1e-8)
        same(a, b, f"call {i} ahead {on}")


def test_ahead_stage_api_and_state_loads():
    spec = (96, 150, 2, 10)
    a = synth(spec, 21, "packed", dict(ypass_ahead=0))
    b = synth(spec, 21, "packed", dict(ypass_ahead=1, handoff_batch=2))
    for f in (a, b):
        f.filter(1e-8)
        f.filter(1e-8)
        # df.cpp:449-461 spelled out: the stage y-pass redoes a set the ahead stream already swept
        f.generate_white_noise()
        for c in range(3):
            f.filtering_sweeps(c)
            f.correlate_fields(c, 1e-8)
        f.apply_RST_scaling()
        f.get_rho_T_fluc()
        f.filter(1e-8)
    same(a, b, "stage api")
    st = a.rng_state()
    for f in (a, b):  # a loaded state discards the prefetched (and swept) noise
        f.set_rng_state(*st)
        f.filter(1e-8)
        f.filter(1e-5)
    same(a, b, "state load")


@pytest.mark.parametrize("ghost", [0, 1])
def test_ahead_strip_groups(ghost):
    Ny, Nz, lo, hi = 80, 900, 4, 32
    o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=23)
    hs = dfamd.create_group(4, tuning=dict(AHEAD, halo_ghost=ghost), plane="synthetic", Ny=Ny, Nz=Nz, N_min=lo,
                            N_max=hi, seed=23, device=0, coeff_mode="table")
    for i in range(5):
        o.filter(1e-8)
        dfamd.filter_group(hs, 1e-8)
        assert all(h.rng_state() == o.rng.state for h in hs), i
        for k in FIELDS:
            got = np.concatenate([h.field(k) for h in hs], axis=1)
            assert np.array_equal(got, o.field(k)), (i, k)


def test_ahead_profile_reports_the_ypass():
    g = synth((256, 512, 4, 32), 3, "table", AHEAD)
    g.set_profiling(True)
    for _ in range(12):
        g.filter(1e-8)
    p = g.profile()
    assert p["calls"] == 12
    assert p["ypass_ms"] > 0 and p["zpass_ms"] > 0, p
