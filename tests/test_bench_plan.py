"""bench.py's multi-GPU workload plan (CPU): the plane and z-strips each N times, checked against the
library's own partition (host-only handles, df_capi.cpp plan_strips), and the whole-job summary
(max-over-ranks time, halo and collective accounting) on synthetic per-rank records."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))

import bench  # noqa: E402


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("name,Ny,Nz", [("c3", 2048, 2048), ("c4", 2048, 8192), ("c5", 4096, 4096)])
def test_strong_plan_matches_library_partition(world, name, Ny, Nz):
    import dfamd
    wl = bench.plan_workload(name, world, "strong")
    assert (wl["Ny"], wl["Nz"]) == (Ny, Nz)  # BASELINE configs[2..4]: the plane does not grow with N
    assert wl["strips"][0][0] == 0 and wl["strips"][-1][1] == Nz
    assert all(a[1] == b[0] for a, b in zip(wl["strips"], wl["strips"][1:]))
    for r in sorted({0, world // 2, world - 1}):
        h = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=4, N_max=64, seed=1, device=-1,
                                rank=r, world=world)
        assert (h.z0, h.z1) == tuple(wl["strips"][r])
        assert h.z1 - h.z0 >= h.comp_info(0)["Nz_max"]  # the halo comes from one neighbour
        h.close()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_weak_plan_gives_each_rank_the_config_plane(world):
    wl = bench.plan_workload("c3", world, "weak")
    assert wl["Nz"] == 2048 * world
    assert all(z1 - z0 == 2048 for z0, z1 in wl["strips"])
    assert wl["scaling"] == ("weak" if world > 1 else "strong")


def test_default_configs():
    a = bench.parse([])
    assert a.config == "auto" and a.scaling == "strong" and a.parity == "on"
    # auto resolves to c3 on one GPU and c4 over N > 1 (main() does exactly this)
    assert bench.plan_workload("c3", 1)["desc"].startswith("c3")
    assert bench.plan_workload("c4", 8)["strips"][7] == (7168, 8192)
    with pytest.raises(ValueError):
        bench.plan_workload("c2", 64)  # 8-column strips are narrower than N_max = 32
    with pytest.raises(ValueError):
        bench.plan_workload("native", 2)


def _rec(rank, el, halo, dom_ms, frac, comm):
    return {"rank": rank, "elapsed_s": el, "columns": [rank * 1024, (rank + 1) * 1024],
            "phase_ms_per_call": {"rng_ms": 0.2, "ypass_ms": 0.8, "halo_ms": halo, "zpass_ms": 0.9, "total_ms": 1.8},
            "roofline": {"avg_launch_ms": dom_ms, "frac": frac, "kernel": "zpass_kernel"}, "comm": comm,
            "call_bytes": 1.0}


def test_summary_takes_the_slowest_rank():
    args = bench.parse(["--steps", "10"])
    wl = bench.plan_workload("c4", 2)
    comm = {"rccl_ranks": 2, "rng_collective": 0, "halo_bytes_sent": 3145728, "rng_bytes_received": 0}

    class Ctx:
        world = 2
    recs = [_rec(0, 0.020, 0.03, 0.9, 0.75, comm), _rec(1, 0.022, 0.05, 0.95, 0.71, comm)]
    s = bench.summarize(Ctx, wl, args, recs)
    assert s["value"] == pytest.approx(2048 * 8192 * 10 / 0.022, rel=1e-6)
    assert s["ms_per_step"] == pytest.approx(2.2)
    mg = s["multi_gpu"]
    assert mg["rccl_ranks"] == 2 and mg["rng_collective"].startswith("none")
    assert mg["rank_ms_per_step"] == {"min": 2.0, "max": 2.2}
    assert mg["halo_ms_per_call"] == {"max": 0.05, "min": 0.03}
    assert mg["halo_bytes_per_call"] == 2 * 3145728 and mg["rng_collective_bytes_per_call"] == 0
    assert s["roofline"]["rank"] == 1 and s["roofline"]["frac_by_rank"] == [0.75, 0.71]


def test_summary_adds_the_whole_call_hbm_figure_for_packed_lines():
    # roofline.call: every rank's algorithmic call bytes over the slowest rank's wall per call (packed only)
    class Ctx:
        world = 2
    wl = bench.plan_workload("c4", 2)
    comm = {"rccl_ranks": 2, "rng_collective": 0, "halo_bytes_sent": 0, "rng_bytes_received": 0}
    recs = [_rec(0, 0.020, 0.03, 0.9, 0.75, comm), _rec(1, 0.022, 0.05, 0.95, 0.71, comm)]
    for r in recs:
        r["call_bytes"] = 5.5e9
    s = bench.summarize(Ctx, wl, bench.parse(["--steps", "10"]), recs)
    call = s["roofline"]["call"]
    assert call["bytes"] == 11e9 and call["ms"] == pytest.approx(2.2)
    assert call["achieved"] == pytest.approx(11e9 / 2.2e-3 / 1e9, rel=1e-4)
    # both ranks' bytes over both ranks' peak (one GPU's peak overstated it N times)
    assert call["frac"] == pytest.approx(call["achieved"] / (2 * bench.HBM_PEAK_GBPS), rel=1e-3)
    t = bench.summarize(Ctx, wl, bench.parse(["--steps", "10", "--coeff-mode", "table"]), recs)
    assert "call" not in t["roofline"]  # the byte model prices the packed stream only
    # table-mode multi-GPU lines keep their multi_gpu block (halo, RNG collective, per-rank times)
    assert t["multi_gpu"]["rccl_ranks"] == 2 and len(t["multi_gpu"]["per_rank"]) == 2


def test_single_gpu_summary_has_no_multi_gpu_block():
    class Ctx:
        world = 1
    wl = bench.plan_workload("c3", 1)
    rec = _rec(0, 0.020, 0.0, 1.7, 0.78, None)
    rec["call_bytes"] = 21.26e9
    s = bench.summarize(Ctx, wl, bench.parse(["--steps", "10"]), [rec])
    assert "multi_gpu" not in s
    assert s["roofline"]["call"]["frac"] == pytest.approx(s["roofline"]["call"]["achieved"] / bench.HBM_PEAK_GBPS,
                                                          rel=1e-3)
