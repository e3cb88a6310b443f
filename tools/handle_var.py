#!/usr/bin/env python3
"""Per-handle spread of the packed sweeps: K c3 handles alive at once, each timed over several rounds in
turn (profiling on: per-phase hipEvents). Prints one JSON line per handle per round."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
import torch  # noqa: E402,F401
import dfamd  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
hs = []
for i in range(K):
    f = dfamd.DigitalFilter(plane="synthetic", Ny=2048, Nz=2048, N_min=4, N_max=64, seed=1, device=0, coeff_mode="packed")
    f.set_profiling(True)
    hs.append(f)
for rnd in range(3):
    for i, f in enumerate(hs):
        f.filter(1e-8)
        f.sync()
        p0 = f.profile()
        for _ in range(8):
            f.filter(1e-8)
        f.sync()
        p1 = f.profile()
        n = p1["calls"] - p0["calls"]
        print(json.dumps({"round": rnd, "handle": i, **{k: round((p1[k] - p0[k]) / n, 4) for k in ("ypass_ms", "zpass_ms", "total_ms")}}), flush=True)
