"""CPU tests of the product's host logic through the C ABI (host-only handles,
device = -1): setup rows, half-widths, coefficients, offsets, stream geometry
and z-strip planning, checked against the reference's golden vectors and the
oracle. No GPU is touched."""
import json
import os

import numpy as np
import pytest

import dfamd
import oracle as O
from conftest import GOLDEN

ROWS8 = ("R11", "R21", "R22", "R33", "Us", "Ts", "rhos", "Ms")


def host(**kw):
    return dfamd.DigitalFilter(device=-1, seed=1, **kw)


def test_library_exports_every_header_symbol():
    L = dfamd.lib()
    syms = dfamd.header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert L.df_abi_version() == 1


def test_native_setup_matches_reference():
    g = np.load(os.path.join(GOLDEN, "native_s42.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "native_s42.json")))
    f = host()
    assert (f.Ny, f.Nz) == (meta["Ny"], meta["Nz"])
    assert f.scalar("u_tau") == meta["u_tau"] and f.scalar("tau_w") == meta["tau_w"]
    for r in ROWS8:
        assert np.array_equal(f.row(r), g["row_" + r]), r
    for c, n in enumerate("uvw"):
        info = f.comp_info(c)
        assert info["Ny_max"] == meta["Ny_max"][c] and info["Nz_max"] == meta["Nz_max"][c]
        assert info["by_size"] == meta["by_size"][c] and info["bz_size"] == meta["bz_size"][c]
        assert np.array_equal(f.halfwidths(c, "y")[:, 0], g["Ny_" + n])
        assert np.array_equal(f.halfwidths(c, "z")[:, 0], g["Nz_" + n])


@pytest.mark.parametrize("name", ["c1_s42", "ramp256_s1234", "ragged_s7"])
def test_synthetic_setup_matches_reference(name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    f = host(plane="synthetic", Ny=int(g["Ny"]), Nz=int(g["Nz"]), N_min=int(g["N_min"]), N_max=int(g["N_max"]))
    for r in ROWS8:
        assert np.array_equal(f.row(r), g["row_" + r]), r
    for c, n in enumerate("uvw"):
        assert np.array_equal(f.halfwidths(c, "y")[:, 0], g["Ny_" + n])
        assert np.array_equal(f.halfwidths(c, "z")[:, 0], g["Nz_" + n])


@pytest.mark.parametrize("spec", [dict(), dict(plane="synthetic", Ny=64, Nz=40, N_min=2, N_max=12)])
def test_coefficients_offsets_and_stream_match_oracle(spec):
    f = host(**spec)
    kw = {}
    if spec:
        kw = dict(plane=O.PLANE_SYNTHETIC, Ny=spec["Ny"], Nz=spec["Nz"], N_min=spec["N_min"], N_max=spec["N_max"])
    o = O.Filter(seed=1, **kw)
    n = o.Ny * o.Nz
    for c in range(3):
        F = o.comp(c)
        by = np.ctypeslib.as_array(F.by, shape=(F.by_size,))
        bz = np.ctypeslib.as_array(F.bz, shape=(F.bz_size,))
        assert np.array_equal(f.coeffs(c, "y"), by)
        assert np.array_equal(f.coeffs(c, "z"), bz)
        assert np.array_equal(f.offsets(c, "y").ravel(), np.ctypeslib.as_array(F.by_offsets, shape=(n,)))
        assert np.array_equal(f.offsets(c, "z").ravel(), np.ctypeslib.as_array(F.bz_offsets, shape=(n,)))
    assert f.stream_length() == sum(O.stream_lengths(o))


def test_coefficients_are_unit_energy():
    # Implicit invariant of df.cpp:166-177: sum_i b_i^2 == 1 for every cell.
    f = host(plane="synthetic", Ny=32, Nz=4, N_min=2, N_max=64)
    for c in range(3):
        b = f.coeffs(c, "y")
        N = f.halfwidths(c, "y").ravel()
        pos = 0
        for n in N:
            seg = b[pos:pos + 2 * n + 1]
            assert abs((seg * seg).sum() - 1.0) < 1e-13
            assert np.array_equal(seg, seg[::-1])
            pos += 2 * n + 1


@pytest.mark.parametrize("world", [2, 3, 8])
def test_strip_partition_covers_plane(world):
    Nz = 1000
    strips = [dfamd.DigitalFilter(device=-1, seed=1, plane="synthetic", Ny=16, Nz=Nz, N_min=2, N_max=8,
                                  rank=r, world=world) for r in range(world)]
    z = [(s.z0, s.z1) for s in strips]
    assert z[0][0] == 0 and z[-1][1] == Nz
    assert all(z[i][1] == z[i + 1][0] for i in range(world - 1))
    assert max(b - a for a, b in z) - min(b - a for a, b in z) <= 1
    whole = host(plane="synthetic", Ny=16, Nz=Nz, N_min=2, N_max=8)
    for c in range(3):
        assert sum(s.comp_info(c)["by_size"] for s in strips) == whole.comp_info(c)["by_size"]
    # every strip draws the same stream: the RNG is replicated, not split
    assert {s.stream_length() for s in strips} == {whole.stream_length()}


def test_strip_narrower_than_halfwidth_is_rejected():
    with pytest.raises(dfamd.DFError, match="narrower"):
        dfamd.DigitalFilter(device=-1, seed=1, plane="synthetic", Ny=16, Nz=20, N_min=2, N_max=16, rank=0, world=4)


def test_bad_inputs_fail_fast(tmp_path):
    with pytest.raises(dfamd.DFError, match="cannot open"):
        host(rst_file=str(tmp_path / "missing.dat"))
    bad = tmp_path / "bad.dat"
    bad.write_text("VARIABLES=x\nZONE f=point\n1 2 3\n")
    with pytest.raises(dfamd.DFError, match="i="):
        host(rst_file=str(bad))
    with pytest.raises(dfamd.DFError, match="synthetic"):
        host(plane="synthetic", Ny=1, Nz=4, N_min=2, N_max=4)


def test_host_only_handle_refuses_gpu_calls():
    f = host()
    with pytest.raises(dfamd.DFError, match="host-only"):
        f.filter(1e-8)


def test_c_abi_rejects_bad_arguments():
    import ctypes as C
    L = dfamd.lib()
    assert L.df_filter(None, 1e-8) == -1
    assert b"null handle" in L.df_last_error()
    f = host()
    assert L.df_get_halfwidths(f._h, 3, 0, None) == -1
    assert L.df_get_row(f._h, 99, (C.c_double * f.Ny)()) == -1
    assert L.df_get_coeffs(f._h, 0, 0, (C.c_double * 4)(), 4) == -1  # too small
    assert "too small" in L.df_last_error().decode()
    assert L.df_set_field(f._h, 5, (C.c_double * 4)()) == -1  # host-only handle
    assert b"host-only" in L.df_last_error()
    assert L.df_set_tuning(None, b"rows_per_wave", 2) == -1
    assert L.df_set_tuning(f._h, b"bogus", 2) == -1
    assert b"unknown tuning" in L.df_last_error()
    assert L.df_set_tuning(f._h, b"rows_per_wave", 2) == 0
    # launch-shape keys that rebalance device tile lists must not touch the absent device state
    # (a host-only handle never built its tap ranges)
    for key in (b"ycoop_order", b"ycoop"):
        assert L.df_set_tuning(f._h, key, 7) == 0
    native = host()  # the reference's grid: long y chains, the row-pair plan
    # the dispatch order re-plans device tables only on handles that have them
    for key, val in ((b"ycoop_order", 4), (b"ycoop_order", 0), (b"yunroll", 8), (b"halo_overlap", 0),
                     (b"halo_overlap", -1), (b"gen_dense", 2), (b"gen_dense", 0), (b"fused_exchange", 0)):
        assert L.df_set_tuning(native._h, key, val) == 0, key
    assert L.df_set_tuning(native._h, b"ycoop_order", -1) == -1
    assert L.df_set_tuning(native._h, b"gen_dense", 1) == -1  # round 5: Kc + K3a removed
    # variants measured neutral or slower are gone from the library, not just off (round 4; round 5: the
    # table y-pass's shared-kernel forms, K3a's destinations switch, the z unroll / store / balance knobs)
    for key in (b"ycoop_map", b"ypre", b"zocc", b"graph", b"count_grid", b"dense_g", b"gen_compact", b"nt_loads",
                b"heavy_first", b"ylds_nw", b"ylds_ch", b"ydepth", b"ywindow", b"ydeep", b"k3a_fast", b"zunroll",
                b"ycoop_ovh", b"znt_stores", b"ynt_stores", b"rng_nt_stores"):
        assert L.df_set_tuning(native._h, key, 1) == -1, key
        assert b"unknown tuning" in L.df_last_error()
    assert L.df_set_tuning(native._h, b"ycoop", 3) == -1
    cfg, keep = dfamd.make_config(device=-1, seed=1, coeff_mode="packed")
    cfg.coeff_mode = 7
    assert not L.df_create(C.byref(cfg))
    assert b"coeff_mode" in L.df_last_error()
    cfg, keep = dfamd.make_config(device=-1, seed=1, rows_per_wave=3)
    assert not L.df_create(C.byref(cfg))
    cfg, keep = dfamd.make_config(device=-1, seed=1, rank=2, world=2)
    assert not L.df_create(C.byref(cfg))


def test_reference_defaults_in_config():
    import ctypes as C
    cfg = dfamd._Cfg()
    dfamd.lib().df_config_default(C.byref(cfg))
    # df.cpp:7-10 hard-coded values
    assert (cfg.d_i, cfg.rho_e, cfg.U_e, cfg.mu_e) == (0.0013, 0.044, 869.1, 7.1212e-6)
    assert cfg.seed_from_random_device == 1 and cfg.plane == 0 and cfg.world == 1
    # drop-in extensions: table mode (bit-identical to packed) and the profiles next to the library
    assert cfg.coeff_mode == dfamd.COEFF["table"]
    dfamd.lib().df_data_dir.restype = C.c_char_p
    data = dfamd.lib().df_data_dir().decode()
    assert os.path.samefile(data, dfamd.DATA)
    assert cfg.vel_fluc_file.decode() == data + "/RST.dat" and cfg.line_file.decode() == data + "/line.dat"


def test_default_config_creates_the_native_plane():
    # an untouched df_config_c (no paths set by the caller) finds its input profiles by itself
    import ctypes as C
    cfg = dfamd._Cfg()
    dfamd.lib().df_config_default(C.byref(cfg))
    cfg.device = -1
    h = dfamd.lib().df_create(C.byref(cfg))
    assert h, dfamd.lib().df_last_error().decode()
    f = dfamd.DigitalFilter(_handle=h)
    assert (f.Ny, f.Nz) == (510, 400)
    f.close()


def test_d_i_from_config_changes_the_setup():
    # the reference ignores DFConfig (df.cpp:7); here d_i scales the grid and length scales
    a = host(plane="synthetic", Ny=32, Nz=8, N_min=2, N_max=8)
    b = dfamd.DigitalFilter(device=-1, seed=1, plane="synthetic", Ny=32, Nz=8, N_min=2, N_max=8, d_i=0.002)
    assert not np.array_equal(a.row("yc"), b.row("yc"))
    assert np.allclose(b.row("yc") / a.row("yc"), 0.002 / 0.0013)


# ---------------------------------------------------------------- grid planes

def _grid_golden():
    return np.load(os.path.join(GOLDEN, "grid_s3.npz"))


def test_grid_plane_setup_matches_reference():
    g = _grid_golden()
    f = dfamd.DigitalFilter(device=-1, seed=1, plane="grid", grid_y=g["grid_y"], grid_z=g["grid_z"])
    assert (f.Ny, f.Nz) == (int(g["Ny"]), int(g["Nz"]))  # RST truncation (df.cpp:280-288)
    assert f.plane_info() == (2, True)
    for r in ROWS8:
        assert np.array_equal(f.row(r), g["row_" + r]), r
    for c, n in enumerate("uvw"):  # per-cell half-widths of the reference's calculate_filter_properties
        assert np.array_equal(f.halfwidths(c, "y"), g["Ny_" + n]), n
        assert np.array_equal(f.halfwidths(c, "z"), g["Nz_" + n]), n
    o = O.Filter(plane=O.PLANE_GRID, Ny=int(g["Ny_in"]), Nz=int(g["Nz_in"]), grid_y=g["grid_y"],
                 grid_z=g["grid_z"], seed=1)
    n = o.Ny * o.Nz
    for c in range(3):
        F = o.comp(c)
        assert np.array_equal(f.coeffs(c, "y"), np.ctypeslib.as_array(F.by, shape=(F.by_size,)))
        assert np.array_equal(f.coeffs(c, "z"), np.ctypeslib.as_array(F.bz, shape=(F.bz_size,)))
        assert np.array_equal(f.offsets(c, "y").ravel(), np.ctypeslib.as_array(F.by_offsets, shape=(n,)))
        assert np.array_equal(f.offsets(c, "z").ravel(), np.ctypeslib.as_array(F.bz_offsets, shape=(n,)))
    assert f.stream_length() == sum(O.stream_lengths(o))
    y, z = f.grid()
    assert np.array_equal(y, g["grid_y"][: f.Ny + 1]) and np.array_equal(z, g["grid_z"][: f.Ny + 1])


def _write_tecplot_grid(path, gy, gz, y_first=False):
    J, I = gy.shape
    with open(path, "w") as fh:
        names = '"y", "z"' if y_first else '"z", "y"'
        fh.write(f"VARIABLES = {names}, \"u_fluc\", \"v_fluc\", \"w_fluc\" \n")
        fh.write(f'ZONE T="Flow Field", I={I}, J={J}, F=BLOCK\n')
        fh.write("VARLOCATION=([3-5]=CELLCENTERED)\n")
        for a in ((gy, gz) if y_first else (gz, gy)):
            fh.write("\n".join(repr(float(v)) for v in a.ravel()) + "\n")


@pytest.mark.parametrize("y_first", [False, True])
def test_grid_plane_from_tecplot_file(tmp_path, y_first):
    # grid_file (df.hpp:47) in write_tecplot's BLOCK layout (df.cpp:712-762)
    g = _grid_golden()
    p = tmp_path / "grid.dat"
    _write_tecplot_grid(p, g["grid_y"], g["grid_z"], y_first)
    f = dfamd.DigitalFilter(device=-1, seed=1, plane="grid", grid_file=str(p))
    a = dfamd.DigitalFilter(device=-1, seed=1, plane="grid", grid_y=g["grid_y"], grid_z=g["grid_z"])
    assert (f.Ny, f.Nz) == (a.Ny, a.Nz)
    for c in range(3):
        for d in "yz":
            assert np.array_equal(f.halfwidths(c, d), a.halfwidths(c, d))


def test_row_uniform_grid_is_not_per_cell():
    # the reference's own placeholder grid fed back as vertices: per-row N, identical setup
    nat = host()
    y, z = nat.grid()
    f = dfamd.DigitalFilter(device=-1, seed=1, plane="grid", grid_y=y, grid_z=z)
    assert f.plane_info() == (2, False)
    for c in range(3):
        for d in "yz":
            assert np.array_equal(f.halfwidths(c, d), nat.halfwidths(c, d))


def test_grid_plane_rejects_bad_vertices(tmp_path):
    g = _grid_golden()
    bad = g["grid_z"].copy()
    bad[:, 5] = bad[:, 4]  # zero-width column
    with pytest.raises(dfamd.DFError, match="increase"):
        dfamd.DigitalFilter(device=-1, seed=1, plane="grid", grid_y=g["grid_y"], grid_z=bad)
    with pytest.raises(dfamd.DFError, match="grid plane needs"):
        dfamd.DigitalFilter(device=-1, seed=1, plane="grid", Ny=4, Nz=4)
    p = tmp_path / "g.dat"
    p.write_text("VARIABLES = \"z\", \"y\"\nZONE I=3, J=3\n1 2 3\n")
    with pytest.raises(dfamd.DFError, match="fewer values"):
        dfamd.DigitalFilter(device=-1, seed=1, plane="grid", grid_file=str(p))


@pytest.mark.parametrize("world", [2, 3])
def test_grid_plane_strips_partition_coefficients(world):
    g = _grid_golden()
    kw = dict(device=-1, seed=1, plane="grid", grid_y=g["grid_y"], grid_z=g["grid_z"])
    whole = dfamd.DigitalFilter(**kw)
    strips = [dfamd.DigitalFilter(rank=r, world=world, **kw) for r in range(world)]
    for c in range(3):
        for d in "yz":
            assert np.array_equal(np.concatenate([s.halfwidths(c, d) for s in strips], axis=1),
                                  whole.halfwidths(c, d))
        assert sum(s.comp_info(c)["by_size"] for s in strips) == whole.comp_info(c)["by_size"]


def test_alloc_registry_rejects_overlapping_ranges():
    """every device allocation of every handle is checked against the live ranges
    of all handles; an overlap fails with DF_EHIP naming both ranges (fed synthetic ranges here)."""
    import ctypes as C
    L = dfamd.lib()
    L.df_alloc_registry.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    L.df_alloc_registry_count.restype = C.c_longlong
    base = 0x7f0000000000  # far from any host or device mapping of this process; never dereferenced
    n0 = L.df_alloc_registry_count()
    assert L.df_alloc_registry(base, 0x1000, 1) == 0
    assert L.df_alloc_registry(base + 0x1000, 0x1000, 1) == 0  # adjacent: no overlap
    assert L.df_alloc_registry_count() == n0 + 2
    for start, size in ((base + 0x800, 0x1000),    # straddles the first range's end
                        (base - 0x10, 0x20),        # straddles the first range's start
                        (base + 0x100, 0x10),       # inside
                        (base - 0x1000, 0x4000)):   # covers both
        assert L.df_alloc_registry(start, size, 1) == -3  # DF_EHIP
        msg = L.df_last_error().decode()
        assert "overlaps the live range" in msg and hex(start) in msg, msg
    assert L.df_alloc_registry_count() == n0 + 2  # a refused claim is not recorded
    assert L.df_alloc_registry(base, 0, 0) == 0 and L.df_alloc_registry(base + 0x1000, 0, 0) == 0
    assert L.df_alloc_registry_count() == n0
    assert L.df_alloc_registry(base + 0x800, 0x1000, 1) == 0  # free again after release
    assert L.df_alloc_registry(base + 0x800, 0, 0) == 0


@pytest.mark.parametrize("plane,mode,expect", [
    # the reference's grid (y half-widths up to 212): table LDS-staged 64-column tiles (ypass_t64), epochs of 4;
    # packed the row-pair y-pass in heaviest-first groups of 4; both with the y-pass ahead on its own stream
    (dict(), "table", dict(rows_per_wave=1, ylds=3, yt_rows=2, yt_chunk=16, handoff_batch=4, ycoop=0, ypass_ahead=1)),
    (dict(), "packed", dict(rows_per_wave=1, ycoop=7, ycoop_order=4, ycoop_split=96, ycoop_split4=192, ylds=0,
                            handoff_batch=4, ypass_ahead=1)),
    # c3 (half-widths 4-64): table 4 rows per wave (ypass_table_kernel), no LDS staging, two generations per
    # hand-off, the run generation; packed 2 rows, one hand-off per call
    (dict(plane="synthetic", Ny=2048, Nz=2048, N_min=4, N_max=64), "table",
     dict(rows_per_wave=4, ylds=0, handoff_batch=2, ycoop=0, gen_dense=2, ypass_ahead=0)),
    (dict(plane="synthetic", Ny=2048, Nz=2048, N_min=4, N_max=64), "packed",
     dict(rows_per_wave=2, ylds=0, ycoop=0, handoff_batch=1, ypass_ahead=0)),
    # c2: epochs of 2; packed: a wave per component in the z-pass
    (dict(plane="synthetic", Ny=512, Nz=512, N_min=4, N_max=32), "table", dict(rows_per_wave=4, ylds=0, handoff_batch=2)),
    (dict(plane="synthetic", Ny=512, Nz=512, N_min=4, N_max=32), "packed",
     dict(rows_per_wave=2, zsplit=1, handoff_batch=2, gen_split=2)),
    (dict(plane="synthetic", Ny=512, Nz=512, N_min=4, N_max=32), "table", dict(gen_split=4)),
    (dict(), "packed", dict(zsplit=0)),
])
def test_launch_plan_defaults(plane, mode, expect):
    # the plane-dependent launch shapes chosen at create time (df_get_tuning on host-only handles): a change to
    # the planning rules shows here before it shows as a slower bench line
    f = host(coeff_mode=mode, **plane)
    got = {k: f.get_tuning(k) for k in expect}
    assert got == expect
    with pytest.raises(dfamd.DFError, match="unknown tuning"):
        f.get_tuning("warp_size")


def test_round5_tuning_keys_validate_on_host_only_handles():
    # the keys added in round 5 (t64 shapes, row-pair halves/quarters, y-pass ahead, ghost columns) are checked
    # and read back without a device: a host-only handle creates no stream and launches nothing
    f = host(coeff_mode="table")  # the reference's grid, row-uniform N: ypass_t64 by default
    assert (f.get_tuning("yt_rows"), f.get_tuning("yt_chunk"), f.get_tuning("yt_pd")) == (2, 16, 2)
    f.set_tuning("yt_rows", 1)
    f.set_tuning("yt_chunk", 24)
    assert (f.get_tuning("yt_chunk"), f.get_tuning("yt_pd")) == (24, 2)
    with pytest.raises(dfamd.DFError, match="yt_pd 4"):
        f.set_tuning("yt_pd", 4)  # built for 1 x 16 only
    f.set_tuning("yt_chunk", 16)
    f.set_tuning("yt_pd", 4)
    f.set_tuning("yt_rows", 2)  # 2 x 16; the prefetch depth drops to 2
    assert (f.get_tuning("yt_rows"), f.get_tuning("yt_chunk"), f.get_tuning("yt_pd")) == (2, 16, 2)
    with pytest.raises(dfamd.DFError, match="yt_rows x yt_chunk"):
        f.set_tuning("yt_chunk", 24)  # 2 x 24 is not built
    for key in ("ycoop_split", "ycoop_split4"):
        with pytest.raises(dfamd.DFError, match=key):
            f.set_tuning(key, -1)
        f.set_tuning(key, 0)
        assert f.get_tuning(key) == 0
    f.set_tuning("ypass_ahead", 0)
    assert f.get_tuning("ypass_ahead") == 0
    f.set_tuning("ypass_ahead", 1)
    assert f.get_tuning("ypass_ahead") == 1
    with pytest.raises(dfamd.DFError, match="halo_ghost"):
        f.set_tuning("halo_ghost", 1)  # a single plane has no neighbours to stand in for
    f.set_tuning("halo_ghost", 0)
    p = host(coeff_mode="packed", plane="synthetic", Ny=64, Nz=300, N_min=2, N_max=12, rank=0, world=2)
    with pytest.raises(dfamd.DFError, match="halo_ghost"):
        p.set_tuning("halo_ghost", 1)  # table mode only
    t = host(coeff_mode="table", plane="synthetic", Ny=64, Nz=300, N_min=2, N_max=12, rank=0, world=2)
    for v in (1, 0, 1):
        t.set_tuning("halo_ghost", v)
        assert t.get_tuning("halo_ghost") == v


def _parametrized(src, func, arg):
    i = src.index(f"def {func}")
    j = src.rindex(f'@pytest.mark.parametrize("{arg}", ', 0, i)
    blk = src[j + len(f'@pytest.mark.parametrize("{arg}", '):i].strip()
    return eval(blk[:-1], {"dict": dict})  # the test file's own literal list


def test_gpu_parity_tuning_sequences_are_accepted():
    # every df_set_tuning sequence the GPU parity tests apply is valid for the plane it is applied to (checked here
    # on host-only handles: a refused key would otherwise surface only on the GPU box, after minutes of queueing)
    src = open(os.path.join(os.path.dirname(__file__), "test_gpu_parity.py")).read()
    for mode, tuning in _parametrized(src, "test_native_grid_bitexact_vs_oracle", "mode,tuning"):
        f = host(coeff_mode=mode)
        for k, v in tuning.items():
            f.set_tuning(k, v)
    i = src.index("def test_runtime_tuning_is_bitexact")
    a = src.index("settings = [", i)
    b = src.index("]\n", a)
    a2 = src.index("settings += [", b)
    b2 = src.index("]\n", a2)
    base = eval(src[a + len("settings = "):b + 1], {"dict": dict})
    extra = eval(src[a2 + len("settings += "):b2 + 1], {"dict": dict})
    for mode in ("packed", "table"):
        f = host(plane="synthetic", Ny=131, Nz=260, N_min=2, N_max=16, coeff_mode=mode)
        for kw in base + (extra if mode == "table" else []):
            for k, v in kw.items():
                f.set_tuning(k, v)


def test_fortran_module_binds_every_c_entry_point():
    # include/digital_filtering.f90's df_c_binding: one bind(C) interface per function df_c.h declares
    import re
    f90 = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "digital_filtering.f90")).read()
    bound = set(re.findall(r'bind\(C, name="(df_\w+)"\)', f90))
    assert [s for s in dfamd.header_symbols() if s not in bound] == []
