#!/usr/bin/env python3
"""Per-GPU cost of an N-way z-strip split, measured on ONE GPU (timing only).

A handle for rank r of N is created with DFAMD_SOLO_STRIP=1 (no RCCL, halos not exchanged,
fields unreadable) so one GPU runs exactly one rank's per-call work: its strip's sweeps plus
the RNG (replicated counting of the whole plane's stream, or split counting of 1/N with the
all-gather replaced by device copies - a lower bound on that option's cost).

    python tools/strip_timing.py [--config c4|c5|weak] [--mode packed|table] [--replicate 0|1] [--ns 1,2,4,8]

c4 = 2048 x 8192 and c5 = 4096 x 4096 split over N (strong, bench.py's N > 1 default);
weak = 2048 x 2048N (every rank a 2048 x 2048 strip). Prints one JSON line per (N, rank).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
os.environ["DFAMD_SOLO_STRIP"] = "1"

p = argparse.ArgumentParser()
p.add_argument("--config", default="c4", choices=["c4", "c5", "weak"])
p.add_argument("--mode", default="packed", choices=["packed", "table"])
p.add_argument("--replicate", type=int, default=1)
p.add_argument("--ns", default="1,2,4,8")
p.add_argument("--calls", type=int, default=20)
p.add_argument("--tune", default="", help="k=v:k=v... df_set_tuning before the warm-up")
p.add_argument("--env", default="", help="K=V:K=V... environment knobs set before the library loads")
a = p.parse_args()
for kv in filter(None, a.env.split(":")):
    os.environ[kv.split("=")[0]] = kv.split("=")[1]
import dfamd  # noqa: E402

for N in [int(x) for x in a.ns.split(",")]:
    Ny, Nz = {"c4": (2048, 8192), "c5": (4096, 4096), "weak": (2048, 2048 * N)}[a.config]
    for rank in sorted({0, N // 2}):
        f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=4, N_max=64, seed=1, device=0,
                                rank=rank, world=N, coeff_mode=a.mode)
        f.set_tuning("rng_replicate", a.replicate)
        for kv in filter(None, a.tune.split(":")):
            f.set_tuning(kv.split("=")[0], int(kv.split("=")[1]))
        for _ in range(3):
            f.filter(1e-8)
        f.sync()
        f.set_profiling(True)
        t0 = time.perf_counter()
        for _ in range(a.calls):
            f.filter(1e-8)
        f.sync()
        wall = (time.perf_counter() - t0) * 1e3 / a.calls
        pr = f.profile()
        ci = f.comm_info()
        f.close()
        print(json.dumps({"config": a.config, "mode": a.mode, "replicate": a.replicate, "tune": a.tune, "N": N, "rank": rank,
                          "wall_ms": round(wall, 4),
                          **{k: round(pr[k] / pr["calls"], 4) for k in ("rng_ms", "ypass_ms", "zpass_ms", "total_ms")},
                          "rng_blocks_counted": ci["rng_blocks_counted"]}), flush=True)
