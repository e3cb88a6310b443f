#!/usr/bin/env python3
"""Per-GPU cost of an N-way z-strip split, measured on ONE GPU (timing only).

A handle for rank r of N is created with DFAMD_SOLO_STRIP=1 (no RCCL, halos not
exchanged, fields meaningless) so one GPU runs exactly the per-rank work of the
weak-scaling bench (2048 x 2048 per GPU): its strip's sweeps plus the replicated
RNG of the whole 2048 x 2048N plane. Prints ms/call per (N, rank)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
os.environ["DFAMD_SOLO_STRIP"] = "1"
import dfamd  # noqa: E402

res = {}
for N, rank in [(1, 0), (2, 0), (4, 1), (8, 0), (8, 3)]:
    f = dfamd.DigitalFilter(plane="synthetic", Ny=2048, Nz=2048 * N, N_min=4, N_max=64, seed=1, device=0,
                            rank=rank, world=N, coeff_mode=sys.argv[1] if len(sys.argv) > 1 else "packed")
    for _ in range(3):
        f.filter(1e-8)
    f.sync()
    f.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(20):
        f.filter(1e-8)
    f.sync()
    wall = (time.perf_counter() - t0) * 1e3 / 20
    p = f.profile()
    res[f"N{N}_r{rank}"] = {"wall_ms": round(wall, 4), "rng_ms": round(p["rng_ms"] / p["calls"], 4),
                            "ypass_ms": round(p["ypass_ms"] / p["calls"], 4),
                            "zpass_ms": round(p["zpass_ms"] / p["calls"], 4)}
    f.close()
    print(json.dumps({f"N{N}_r{rank}": res[f"N{N}_r{rank}"]}), flush=True)
