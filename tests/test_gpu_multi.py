"""Multi-process z-strips over RCCL, one process and one GPU per rank.

Each rank runs the product's peer path - ncclCommInitRank, the grouped ncclSend/ncclRecv halo
with rank +- 1 (df_capi.cpp phase_halo_rccl) and, with rng_replicate 0, the share records of the
split counting (inside the halo group, or all-gathered) - then compares its strip with the whole plane run unsplit on its own
GPU, bit for bit (fields, filt_old and the stream state). World 1 runs on any box (a one-rank
communicator: the same init and calls, no peers); larger worlds are skipped below that many GPUs.

Emulated hosts (any box with one GPU): every rank runs on device 0 and gets its own NCCL_HOSTID, so
RCCL sees one GPU per "host" (its duplicate-GPU check compares bus ids within a host only) and
connects the ranks through its socket transport over the loopback interface. The product's code is
the same as on an 8-GPU node - the communicator init, the rank +- 1 grouped send/recv, the halo
pack/unpack and the all-gather - only RCCL's transport underneath differs (socket, not xGMI).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "mgpu_worker.py")


def n_gpus():
    import torch
    return torch.cuda.device_count()  # does not initialise the GPU on this image


def emulated_host_env(rank):
    """Environment that makes RCCL treat this process as the only GPU of its own host."""
    return dict(os.environ, NCCL_HOSTID=f"dfamd-emulated-host-{rank}", NCCL_SOCKET_IFNAME="lo",
                NCCL_IB_DISABLE="1", NCCL_NET="Socket", HSA_ENABLE_IPC_MODE_LEGACY="0")


def run_world(world, mode, replicate, Ny=256, Nz=1024, N_min=4, N_max=32, seed=11, dts=(1e-8, 1e-8, 1e-5),
              emulate=False, extra=None):
    sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
    import dfamd
    cid = dfamd.comm_unique_id().hex()  # the bootstrap root lives in this process until the ranks join
    procs = []
    for r in range(world):
        spec = dict(rank=r, world=world, comm_id=cid, Ny=Ny, Nz=Nz, N_min=N_min, N_max=N_max, seed=seed,
                    mode=mode, replicate=replicate, dts=list(dts), device=0 if emulate else r, **(extra or {}))
        procs.append(subprocess.Popen([sys.executable, WORKER, json.dumps(spec)], stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, start_new_session=True,
                                      env=emulated_host_env(r) if emulate else None))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=150)
            assert p.returncode == 0, f"rank exited {p.returncode}: {e[-2000:]}"
            outs.append(json.loads(o.strip().splitlines()[-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
                p.wait()
    return outs


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("mode,replicate", [("packed", 1), ("table", 1), ("packed", 0), ("table", 0)])
def test_rccl_strips_match_unsplit_plane(world, mode, replicate):
    if n_gpus() < world:
        pytest.skip(f"needs {world} GPUs, box has {n_gpus()}")
    outs = run_world(world, mode, replicate)
    check_world(outs, world, replicate)


def check_world(outs, world, replicate, Nz=1024, ghost=False):
    cols = sorted(o["columns"] for o in outs)
    assert cols[0][0] == 0 and cols[-1][1] == Nz
    assert all(a[1] == b[0] for a, b in zip(cols, cols[1:]))
    for o in outs:
        assert o["mismatch"] == {}, o
        assert o["rng_equal"], o
        c = o["comm"]
        assert c["rccl_ranks"] == world
        assert c["rng_collective"] in ((0,) if replicate else (1, 2))  # 2: records in the halo group
        assert c["halo_peers"] == (0 if world == 1 or ghost else (1 if o["rank"] in (0, world - 1) else 2))


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("mode,replicate", [("packed", 1), ("table", 1), ("table", 0), ("packed", 0)])
def test_rccl_strips_emulated_hosts(world, mode, replicate):
    """world ranks on one GPU, one emulated host each: the peer send/recv path on a one-GPU box."""
    if n_gpus() < 1:
        pytest.skip("needs a GPU")
    outs = run_world(world, mode, replicate, emulate=True)
    check_world(outs, world, replicate)


@pytest.mark.parametrize("world,Nz", [(2, 1024), (3, 1000), (4, 2048)])
@pytest.mark.parametrize("mode,replicate", [("packed", 1), ("table", 0)])
@pytest.mark.parametrize("overlap", [0, 1])
def test_rccl_halo_overlap_forms_emulated(world, Nz, mode, replicate, overlap):
    """Both halo forms bit-equal to the unsplit plane: the exchange under the interior strips' z-pass (the
    default; N_max 64 leaves 1-3 interior strips per rank here) and the serial chain (halo_overlap 0)."""
    if n_gpus() < 1:
        pytest.skip("needs a GPU")
    outs = run_world(world, mode, replicate, Nz=Nz, N_min=4, N_max=64, emulate=True,
                     extra=dict(halo_overlap=overlap))
    check_world(outs, world, replicate, Nz=Nz)


@pytest.mark.parametrize("mode,replicate,tuning", [("packed", 1, {}), ("table", 0, {}), ("table", 0, {"gen_dense": 2})])
def test_rccl_c4_real_partition_emulated(mode, replicate, tuning):
    """The partition the driver's 8-GPU bench runs first: BASELINE configs[3] (c4,
    2048 x 8192, N 4-64) in eight 2048 x 1024 strips, each rank's 2.5 MB halos per side through the
    product's grouped ncclSend/ncclRecv (RCCL socket transport between emulated hosts on one GPU), every
    strip bit-equal to the whole plane run unsplit after step 0 and two calls."""
    if n_gpus() < 1:
        pytest.skip("needs a GPU")
    outs = run_world(8, mode, replicate, Ny=2048, Nz=8192, N_min=4, N_max=64, dts=(1e-8, 1e-5), emulate=True,
                     extra=dict(tuning=tuning))
    check_world(outs, 8, replicate, Nz=8192)
    assert sorted(o["columns"] for o in outs) == [[r * 1024, (r + 1) * 1024] for r in range(8)]
    # the halo of row j carries that row's widest z half-width (not N_max) columns per side
    import numpy as np
    import dfamd
    host = dfamd.DigitalFilter(plane="synthetic", Ny=2048, Nz=8192, N_min=4, N_max=64, seed=11, device=-1,
                               coeff_mode=mode)
    per_side = 8 * sum(int(np.minimum(host.halfwidths(c, "z").max(axis=1), host.comp_info(c)["Nz_max"]).sum())
                       for c in range(3))
    assert per_side < 2048 * 64 * 3 * 8
    for o in outs:
        assert o["comm"]["halo_bytes_sent"] == o["comm"]["halo_peers"] * per_side, (o["comm"], per_side)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("fused", [1, 0])
def test_rccl_run_generation_emulated(world, fused):
    """Table mode with split counting and the run generation (gen_dense 2): the group counts of the next
    generation travel inside the call's halo group (fused_exchange 1, one grouped RCCL operation per call) or
    in an all-gather of their own (0); every strip bit-equal to the unsplit plane."""
    if n_gpus() < 1:
        pytest.skip("needs a GPU")
    outs = run_world(world, "table", 0, emulate=True, extra=dict(tuning=dict(gen_dense=2, fused_exchange=fused)))
    check_world(outs, world, 0)
    assert all(o["comm"]["rng_collective"] == (2 if fused else 1) for o in outs)
    for o in outs:  # each other rank's share record: 64 group counts + an int32 prefix per block, an int64 total
        chunk = o["comm"]["rng_blocks_counted"]
        rec = ((chunk * 68 + 7) // 8 * 8 + 8 + 15) // 16 * 16
        assert o["comm"]["rng_bytes_received"] == rec * (world - 1)


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("fused", [1, 0])
def test_rccl_halo_ghost_emulated(world, fused):
    """Ghost columns (halo_ghost 1, round 5): no halo send/recv at all - each rank y-filters its neighbours'
    halo columns itself - and the share records all-gathered on the RNG stream (fused 1: right after the
    counts; 0: the plain per-generation all-gather); every strip bit-equal to the unsplit plane."""
    if n_gpus() < 1:
        pytest.skip("needs a GPU")
    outs = run_world(world, "table", 0, Nz=1024, N_min=4, N_max=64, emulate=True,
                     extra=dict(tuning=dict(gen_dense=2, fused_exchange=fused, halo_ghost=1)))
    check_world(outs, world, 0, ghost=True)
    for o in outs:
        assert o["comm"]["halo_bytes_sent"] == 0 and o["comm"]["halo_peers"] == 0, o["comm"]
        assert o["comm"]["rng_collective"] == 1, o["comm"]


def test_rccl_c4_real_partition_ghost_emulated():
    """c4 (2048 x 8192, N 4-64) in eight strips with ghost columns: every strip bit-equal to the whole plane."""
    if n_gpus() < 1:
        pytest.skip("needs a GPU")
    outs = run_world(8, "table", 0, Ny=2048, Nz=8192, N_min=4, N_max=64, dts=(1e-8, 1e-5), emulate=True,
                     extra=dict(tuning=dict(gen_dense=2, halo_ghost=1)))
    check_world(outs, 8, 0, Nz=8192, ghost=True)
