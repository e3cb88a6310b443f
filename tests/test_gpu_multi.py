"""Multi-process z-strips over RCCL, one process and one GPU per rank.

Each rank runs the product's peer path - ncclCommInitRank, the grouped ncclSend/ncclRecv halo
with rank +- 1 (df_capi.cpp phase_halo_rccl) and, with rng_replicate 0, the per-call all-gather
of accept counts and masks - then compares its strip with the whole plane run unsplit on its own
GPU, bit for bit (fields, filt_old and the stream state). World 1 runs on any box (a one-rank
communicator: the same init and calls, no peers); larger worlds are skipped below that many GPUs.
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


def run_world(world, mode, replicate, Ny=256, Nz=1024, N_min=4, N_max=32, seed=11, dts=(1e-8, 1e-8, 1e-5)):
    sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
    import dfamd
    cid = dfamd.comm_unique_id().hex()
    procs = []
    for r in range(world):
        spec = dict(rank=r, world=world, comm_id=cid, Ny=Ny, Nz=Nz, N_min=N_min, N_max=N_max, seed=seed,
                    mode=mode, replicate=replicate, dts=list(dts))
        procs.append(subprocess.Popen([sys.executable, WORKER, json.dumps(spec)], stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, start_new_session=True))
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
@pytest.mark.parametrize("mode,replicate", [("packed", 1), ("table", 1), ("packed", 0)])
def test_rccl_strips_match_unsplit_plane(world, mode, replicate):
    if n_gpus() < world:
        pytest.skip(f"needs {world} GPUs, box has {n_gpus()}")
    outs = run_world(world, mode, replicate)
    cols = sorted(o["columns"] for o in outs)
    assert cols[0][0] == 0 and cols[-1][1] == 1024
    for o in outs:
        assert o["mismatch"] == {}, o
        assert o["rng_equal"], o
        c = o["comm"]
        assert c["rccl_ranks"] == world
        assert c["rng_collective"] == (0 if replicate else 1)
        assert c["halo_peers"] == (0 if world == 1 else (1 if o["rank"] in (0, world - 1) else 2))
