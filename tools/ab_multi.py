#!/usr/bin/env python3
"""In-process timing of several df_set_tuning variants on ONE handle (same allocations), interleaved rounds.

    python3 tools/ab_multi.py --config native --mode table --tune ylds=2,rows_per_wave=1 --tune ylds=3,yt_rows=2

Prints one JSON line per variant: median / min over rounds of the per-phase hipEvent times and the wall time
per call (tools/ab.py's A/B with any number of variants).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
import torch  # noqa: E402,F401  (binds libdfamd to torch's HIP runtime first, as bench.py does)
import dfamd  # noqa: E402

CFG = {"c1": (128, 128, 8, 8), "c2": (512, 512, 4, 32), "c3": (2048, 2048, 4, 64), "c5": (4096, 4096, 4, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="native")
    ap.add_argument("--mode", default="table")
    ap.add_argument("--tune", action="append", default=[])
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--calls", type=int, default=20)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    if a.config == "native":
        f = dfamd.DigitalFilter(plane="native", seed=1, device=0, coeff_mode=a.mode)
    else:
        Ny, Nz, lo, hi = CFG[a.config]
        f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=1, device=0,
                                coeff_mode=a.mode)
    variants = [[(kv.split("=")[0], int(kv.split("=")[1])) for kv in filter(None, t.split(","))] for t in a.tune] or [[]]
    rec = [{p: [] for p in ("rng_ms", "ypass_ms", "zpass_ms", "total_ms", "wall_ms")} for _ in variants]
    for _ in range(3):
        f.filter(1e-8)
    f.sync()
    for _ in range(a.rounds):
        for i, v in enumerate(variants):
            for key, val in v:
                f.set_tuning(key, val)
            f.filter(1e-8)
            f.filter(1e-8)
            f.sync()
            f.set_profiling(True)
            t0 = time.perf_counter()
            for _ in range(a.calls):
                f.filter(1e-8)
            f.sync()
            wall = (time.perf_counter() - t0) * 1e3 / a.calls
            p = f.profile()
            f.set_profiling(False)
            p["wall_ms"] = wall * p["calls"]
            for ph in rec[i]:
                rec[i][ph].append(p[ph] / p["calls"])
    for t, r in zip(a.tune or [""], rec):
        print(json.dumps({"config": a.config, "mode": a.mode, "tune": t,
                          "median_ms": {ph: round(statistics.median(v), 4) for ph, v in r.items()},
                          "min_ms": {ph: round(min(v), 4) for ph, v in r.items()}}))


if __name__ == "__main__":
    main()
