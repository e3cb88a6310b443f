"""Ghost columns (round 5): table-mode z-strips y-filter their strip widened by their
neighbours' halo columns (the plane's widest z half-width each side) straight into their own z-halo, so the
z-pass needs no halo exchange and the only collective left, the RNG share records, runs on the RNG stream two
generations ahead. The ghost columns are the neighbours' own y-filtered columns recomputed from the same
noise (the RNG stores those r_ys columns too), the same products in the same order (df.cpp:359-383): every
strip must equal the unsplit plane and the oracle bit for bit, and the stream state must match after every
call. In-process strip groups here; the RCCL form in tests/test_gpu_multi.py."""
import numpy as np
import pytest

import dfamd
import oracle as O

pytestmark = pytest.mark.gpu
FIELDS = ("u", "v", "w", "T", "rho")
GHOST = dict(halo_ghost=1)


def check(hs, o, what):
    assert all(h.rng_state() == o.rng.state for h in hs), what
    for k in FIELDS:
        got = np.concatenate([h.field(k) for h in hs], axis=1)
        ref = o.field(k)
        if not np.array_equal(got, ref):
            bad = np.argwhere(got != ref)
            raise AssertionError(f"{what} {k}: {len(bad)} cells differ, first {tuple(bad[0])}")


@pytest.mark.parametrize("world,Ny,Nz,lo,hi", [(2, 96, 300, 4, 16), (3, 64, 700, 2, 24), (4, 100, 1100, 4, 64),
                                              (8, 48, 2048, 4, 64), (3, 37, 197, 2, 10)])
@pytest.mark.parametrize("tuning", [{}, dict(ylds=3, yt_rows=2), dict(ylds=2, rows_per_wave=1),
                                    dict(gen_dense=2, gen_split=1, fuse_plan=0)])
def test_ghost_strips_match_oracle(world, Ny, Nz, lo, hi, tuning):
    o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=19)
    hs = dfamd.create_group(world, tuning=dict(GHOST, **tuning), plane="synthetic", Ny=Ny, Nz=Nz, N_min=lo,
                            N_max=hi, seed=19, device=0, coeff_mode="table")
    assert all(h.get_tuning("halo_ghost") == 1 for h in hs)
    assert all(h.comm_info()["halo_bytes_sent"] == 0 for h in hs)
    check(hs, o, "step0")
    for i, dt in enumerate((1e-8, 1e-8, 1e-5)):
        o.filter(dt)
        dfamd.filter_group(hs, dt)
        check(hs, o, f"call {i}")


def test_ghost_toggled_mid_run_and_noise_arrays():
    # the halo form switched between calls (the prefetched noise is redrawn in the other layout each time), and
    # each strip's own r_ys columns equal the oracle's
    spec = dict(plane="synthetic", Ny=80, Nz=900, N_min=4, N_max=32, seed=23, device=0, coeff_mode="table")
    o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=80, Nz=900, N_min=4, N_max=32, seed=23)
    hs = dfamd.create_group(4, **spec)
    for i, g in enumerate((1, 1, 0, 1, 0, 0, 1)):
        for h in hs:
            h.set_tuning("halo_ghost", g)
        o.filter(1e-8)
        dfamd.filter_group(hs, 1e-8)
        check(hs, o, f"call {i} ghost {g}")
    for c in range(3):
        F = o.comp(c)
        ry = np.ctypeslib.as_array(F.r_ys, shape=(F.r_ys_size,)).reshape(-1, o.Nz)
        got = np.concatenate([h.noise(c, "y") for h in hs], axis=1)
        assert np.array_equal(got, ry), c


def test_ghost_disagreement_is_refused_before_any_strip_draws():
    # a group call whose strips disagree on halo_ghost fails before any strip consumes a generation,
    # so once they agree the run continues in step with the reference
    spec = dict(plane="synthetic", Ny=64, Nz=600, N_min=4, N_max=24, seed=29, device=0, coeff_mode="table")
    o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=64, Nz=600, N_min=4, N_max=24, seed=29)
    hs = dfamd.create_group(3, **spec)
    hs[1].set_tuning("halo_ghost", 1)
    with pytest.raises(dfamd.DFError, match="halo_ghost differs"):
        dfamd.filter_group(hs, 1e-8)
    hs[0].set_tuning("halo_ghost", 1)
    hs[2].set_tuning("halo_ghost", 1)
    for i in range(2):
        o.filter(1e-8)
        dfamd.filter_group(hs, 1e-8)
        check(hs, o, f"call {i} after the refused call")


def test_ghost_needs_table_mode_and_row_uniform_planes():
    packed = dfamd.create_group(2, plane="synthetic", Ny=40, Nz=300, N_min=4, N_max=8, seed=1, device=0,
                                coeff_mode="packed")
    with pytest.raises(dfamd.DFError, match="halo_ghost"):
        packed[0].set_tuning("halo_ghost", 1)
    one = dfamd.DigitalFilter(plane="synthetic", Ny=40, Nz=300, N_min=4, N_max=8, seed=1, device=0,
                              coeff_mode="table")
    with pytest.raises(dfamd.DFError, match="halo_ghost"):
        one.set_tuning("halo_ghost", 1)
    one.set_tuning("halo_ghost", 0)  # off is always accepted
