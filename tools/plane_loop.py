#!/usr/bin/env python3
"""A plane driven for K calls, for rocprofv3 kernel traces and PMC passes of one configuration.
    rocprofv3 ... -- python3 tools/plane_loop.py native|c1|c2|c3|c5 [packed|table] [calls] [key=value tuning ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
import torch  # noqa: E402,F401
import dfamd  # noqa: E402

CFG = {"c1": (128, 128, 8, 8), "c2": (512, 512, 4, 32), "c3": (2048, 2048, 4, 64), "c5": (4096, 4096, 4, 64)}
name = sys.argv[1]
mode = sys.argv[2] if len(sys.argv) > 2 else "packed"
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 10
if name == "native":
    f = dfamd.DigitalFilter(plane="native", seed=1, device=0, coeff_mode=mode)
else:
    Ny, Nz, lo, hi = CFG[name]
    f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=1, device=0, coeff_mode=mode)
for kv in sys.argv[4:]:
    k, v = kv.split("=")
    f.set_tuning(k, int(v))
for _ in range(calls):
    f.filter(1e-8)
f.sync()
