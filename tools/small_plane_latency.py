#!/usr/bin/env python3
"""Per-call latency of small planes, where launches rather than bytes set the time:
the reference's own grid (plane "native", 510 x 400 after truncation) and c1 / c2.
Prints one JSON line per plane: async and synchronous us per filter(dt), plus hipEvent
phase times. Usage: python3 tools/small_plane_latency.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "digital-filtering_amd"))
import torch  # noqa: E402,F401
import dfamd  # noqa: E402

PLANES = [("native", dict(plane="native")), ("c1", dict(plane="synthetic", Ny=128, Nz=128, N_min=8, N_max=8)),
          ("c2", dict(plane="synthetic", Ny=512, Nz=512, N_min=4, N_max=32))]
for name, kw in PLANES:
    for mode in ("packed", "table"):
        f = dfamd.DigitalFilter(seed=1, device=0, coeff_mode=mode, **kw)
        for _ in range(20):
            f.filter(1e-8)
        f.sync()
        t0 = time.perf_counter()
        for _ in range(500):
            f.filter(1e-8)
        f.sync()
        t1 = time.perf_counter()
        for _ in range(200):
            f.filter(1e-8)
            f.sync()
        t2 = time.perf_counter()
        f.set_profiling(True)
        for _ in range(100):
            f.filter(1e-8)
        f.sync()
        p = f.profile()
        print(json.dumps({"plane": name, "mode": mode, "Ny": f.Ny, "Nz": f.Nz,
                          "async_us_per_call": round((t1 - t0) / 500 * 1e6, 1),
                          "sync_us_per_call": round((t2 - t1) / 200 * 1e6, 1),
                          "phase_us": {k: round(p[k] / p["calls"] * 1e3, 1)
                                       for k in ("rng_ms", "ypass_ms", "zpass_ms", "total_ms")}}), flush=True)
        del f
