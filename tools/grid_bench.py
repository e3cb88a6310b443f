#!/usr/bin/env python3
"""Timing of a real-grid plane (per-cell half-widths) on one GPU; not the headline bench.

A warped tanh-stretched grid (oracle.warped_grid) of Ny x Nz cells with physical spacing, so the
half-widths follow df.cpp:144-195 per cell. Prints one JSON line per coefficient mode: ms per
filter(dt), cells/s, and SURVEY 8d algorithmic GB/s of the sweeps (per-cell sum(2N+1); the device
stream additionally holds the zero taps that pad each (strip, row) to its widest cell)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "digital-filtering_amd"), os.path.join(ROOT, "oracle")]
import torch  # noqa: E402,F401
import dfamd  # noqa: E402
import oracle as O  # noqa: E402  (grid generator only)

Ny, Nz = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (512, 2048)
gy, gz = O.warped_grid(Ny, Nz, dz0=2.4e-5, wave=0.12)
for mode in ("packed", "table"):
    f = dfamd.DigitalFilter(plane="grid", grid_y=gy, grid_z=gz, device=0, seed=1, coeff_mode=mode)
    hw = [f.halfwidths(c, d) for c in range(3) for d in "yz"]
    pad = 0
    for c in range(3):
        for d in "yz":
            N = f.halfwidths(c, d)
            ncol = N.shape[1]
            for s0 in range(0, ncol, 128):
                blk = N[:, s0:s0 + 128]
                pad += int(((2 * blk.max(axis=1) + 1) * 128).sum() - (2 * blk + 1).sum())
    for _ in range(5):
        f.filter(1e-8)
    f.sync()
    f.set_profiling(True)
    t0 = time.perf_counter()
    n = 30
    for _ in range(n):
        f.filter(1e-8)
    f.sync()
    ms = (time.perf_counter() - t0) * 1e3 / n
    p = f.profile()
    sweeps = (p["ypass_ms"] + p["zpass_ms"]) / p["calls"]
    alg = f.algorithmic_bytes(-1)
    print(json.dumps({"plane": f"grid {f.Ny}x{f.Nz} (per-cell N)", "mode": mode, "ms_per_call": round(ms, 4),
                      "cells_per_s": round(f.Ny * f.Nz / ms * 1e3, 1),
                      "N_range": [int(min(h.min() for h in hw)), int(max(h.max() for h in hw))],
                      "alg_GB": round(alg / 1e9, 3), "pad_zero_taps_GB": round(pad * 8 / 1e9, 3),
                      "sweeps_ms": round(sweeps, 4),
                      "alg_GBps_sweeps": round(alg / (sweeps * 1e-3) / 1e9, 1) if mode == "packed" else None}))
    f.close()
