#!/usr/bin/env python3
"""BASELINE configs[4] on one GPU: a 4096 x 4096 plane (N 4-64), u'/v'/w' + SRA T'/rho', for
STEPS filter(dt) calls (default 10 000), with the device-side get_rms accumulation every step
(df.cpp:566-611). Reports the time per call and the SURVEY 4 invariant at the end: per row,
mean(u'^2) -> R11, mean(v'^2) -> R22, mean(w'^2) -> R33 (rows with R11 > 1% of its max).
    python3 tools/long_run.py [STEPS] [dt]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
import torch  # noqa: E402,F401
import dfamd  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
dt = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-8
f = dfamd.DigitalFilter(plane="synthetic", Ny=4096, Nz=4096, N_min=4, N_max=64, seed=2026, device=0)
f.filter(dt)
f.sync()
f.rms_reset()
t0 = time.perf_counter()
last = t0
for i in range(steps):
    f.filter(dt)
    f.rms_add()
    if (i + 1) % 1000 == 0:
        f.sync()
        now = time.perf_counter()
        print(json.dumps({"step": i + 1, "ms_per_call_last_1000": round((now - last), 4)}), flush=True)
        last = now
f.sync()
total = time.perf_counter() - t0
R = {k: f.row(k) for k in ("R11", "R22", "R33")}
rows = R["R11"] > 0.01 * R["R11"].max()
dev = {}
for name, r in (("u", "R11"), ("v", "R22"), ("w", "R33")):
    ms = (f.rms(name) ** 2).mean(axis=1)
    dev[name] = float(np.abs(ms[rows] / R[r][rows] - 1).max())
state = f.rng_state()
print(json.dumps({"config": "c5 4096x4096 N 4-64, packed, 1 GPU", "steps": steps, "dt": dt,
                  "total_s": round(total, 2), "ms_per_call_incl_rms": round(total * 1e3 / steps, 3),
                  "rms_count": f.rms_count() if hasattr(f, "rms_count") else steps,
                  "max_rel_dev_rowvar_vs_R": dev, "rows_checked": int(rows.sum()),
                  "fields_finite": bool(all(np.isfinite(f.field(k)).all() for k in ("u", "v", "w", "T", "rho"))),
                  "rng_state": [str(state[0]), state[1]]}))
