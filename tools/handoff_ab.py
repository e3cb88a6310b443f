#!/usr/bin/env python3
"""Wall time per call with the per-call stream hand-off ablated (DFAMD_ABLATE_HANDOFF, timing only:
1 no wait for the noise, 2 no release event, 3 neither), one handle per variant, no phase events.
    python3 tools/handoff_ab.py config mode [rounds] [calls]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
import torch  # noqa: E402,F401
import dfamd  # noqa: E402

cfg, mode = sys.argv[1], sys.argv[2]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 50
dims = {"c1": (128, 128, 8, 8), "c2": (512, 512, 4, 32), "c3": (2048, 2048, 4, 64)}
hs = {}
for v in ("0", "1", "2", "3"):
    os.environ["DFAMD_ABLATE_HANDOFF"] = v
    if cfg == "native":
        hs[v] = dfamd.DigitalFilter(seed=1, device=0, coeff_mode=mode)
    else:
        Ny, Nz, a, b = dims[cfg]
        hs[v] = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=a, N_max=b, seed=1, device=0, coeff_mode=mode)
os.environ.pop("DFAMD_ABLATE_HANDOFF")
res = {v: [] for v in hs}
for f in hs.values():
    for _ in range(30):
        f.filter(1e-8)
    f.sync()
for _ in range(rounds):
    for v, f in hs.items():
        f.sync()
        t0 = time.perf_counter()
        for _ in range(calls):
            f.filter(1e-8)
        f.sync()
        res[v].append((time.perf_counter() - t0) * 1e3 / calls)
print(json.dumps({"config": cfg, "mode": mode, "ms_per_call_median": {v: round(statistics.median(x), 4) for v, x in res.items()}}))
