"""bench.py's N > 1 plumbing over gloo on CPU (world 2 and 4): the RCCL id broadcast from rank 0,
the all-gather of per-rank records, the max-over-ranks summary and the parity vote. The GPU parts
(handles, RCCL) are exercised by tests/test_gpu_multi.py; here a stand-in library object returns
the unique id, so the collective call pattern bench.main() uses is run with real ranks."""
import os
import socket
import sys

import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeLib:
    @staticmethod
    def comm_unique_id():
        return bytes(range(128))


def _worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import bench
    ctx = bench.Ctx()
    ctx.init(torch, backend="gloo")
    cid = ctx.comm_id(_FakeLib)
    args = bench.parse(["--steps", "10", "--gpus", str(world)])
    wl = bench.plan_workload("c4", world)
    z0, z1 = wl["strips"][rank]
    rec = {"rank": rank, "elapsed_s": 0.02 + 0.001 * rank, "columns": [z0, z1],
           "phase_ms_per_call": {"rng_ms": 0.1, "ypass_ms": 0.8, "halo_ms": 0.01 * (rank + 1), "zpass_ms": 0.9,
                                 "total_ms": 1.9},
           "roofline": {"avg_launch_ms": 0.9 + 0.01 * rank, "frac": 0.7, "kernel": "zpass_kernel"},
           "comm": {"rccl_ranks": world, "rng_collective": 0,
                    "halo_bytes_sent": (1 if rank in (0, world - 1) else 2) * 2048 * 64 * 3 * 8,
                    "rng_bytes_received": 0},
           "call_bytes": 1.0}
    recs = ctx.gather(rec)
    summary = bench.summarize(ctx, wl, args, recs)
    votes = ctx.gather({"ok": rank != 99})
    ctx.barrier()
    ctx.dist.destroy_process_group()
    results[rank] = {"cid": cid, "summary": summary, "ranks_seen": [r["rank"] for r in recs],
                     "parity_ok": all(v["ok"] for v in votes)}


@pytest.mark.parametrize("world", [2, 4])
def test_bench_collectives_over_gloo(world):
    port = _free_port()
    with mp.Manager() as m:
        results = m.dict()
        mp.spawn(_worker, args=(world, port, results), nprocs=world, join=True)
        res = dict(results)
    assert sorted(res) == list(range(world))
    for r, out in res.items():
        assert out["cid"] == bytes(range(128))  # every rank got rank 0's id
        assert out["ranks_seen"] == list(range(world))
        assert out["parity_ok"]
        s = out["summary"]
        slow = 0.02 + 0.001 * (world - 1)
        assert s["ms_per_step"] == pytest.approx(slow * 100)  # max over ranks, 10 steps
        assert s["value"] == pytest.approx(2048 * 8192 * 10 / slow)
        mg = s["multi_gpu"]
        assert mg["rccl_ranks"] == world
        assert mg["halo_bytes_per_call"] == (2 * world - 2) * 2048 * 64 * 3 * 8
        assert [p["columns"][0] for p in mg["per_rank"]] == [r * 8192 // world for r in range(world)]
