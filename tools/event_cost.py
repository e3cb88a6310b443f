#!/usr/bin/env python3
"""Cost of bench.py's per-call phase events (df_set_profiling: 6 hipEventRecords per call) on the
wall time of short calls: one handle, interleaved rounds of K calls with profiling off and on.
    python3 tools/event_cost.py [config] [mode] [rounds] [calls]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
import torch  # noqa: E402,F401
import dfamd  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
mode = sys.argv[2] if len(sys.argv) > 2 else "packed"
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 9
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 50
dims = {"c1": (128, 128, 8, 8), "c2": (512, 512, 4, 32), "c3": (2048, 2048, 4, 64)}
if cfg == "native":
    f = dfamd.DigitalFilter(seed=1, device=0, coeff_mode=mode)
else:
    Ny, Nz, a, b = dims[cfg]
    f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=a, N_max=b, seed=1, device=0, coeff_mode=mode)
for _ in range(50):
    f.filter(1e-8)
f.sync()
res = {"off": [], "on": [], "every4": []}
for _ in range(rounds):
    for k in res:
        f.set_profiling(k != "off", every=4 if k == "every4" else 1)
        f.sync()
        t0 = time.perf_counter()
        for _ in range(calls):
            f.filter(1e-8)
        f.sync()
        res[k].append((time.perf_counter() - t0) * 1e3 / calls)
        if k != "off":
            f.profile()
print(json.dumps({"config": cfg, "mode": mode, "calls": calls,
                  "ms_per_call_median": {k: round(statistics.median(v), 4) for k, v in res.items()},
                  "ms_per_call_min": {k: round(min(v), 4) for k, v in res.items()}}))
