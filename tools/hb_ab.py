#!/usr/bin/env python3
"""Wall time per call against the hand-off batch (DFAMD_HANDOFF_BATCH 1, 2, 4 at create), one handle per
variant, interleaved rounds, no phase events.
    python3 tools/hb_ab.py config mode [rounds] [calls]"""
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
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 48
dims = {"c1": (128, 128, 8, 8), "c2": (512, 512, 4, 32), "c3": (2048, 2048, 4, 64)}
hs = {}
for v in ("1", "2", "4"):
    os.environ["DFAMD_HANDOFF_BATCH"] = v.rstrip("b")
    if cfg == "native":
        hs[v] = dfamd.DigitalFilter(seed=1, device=0, coeff_mode=mode)
    else:
        Ny, Nz, a, b = dims[cfg]
        hs[v] = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=a, N_max=b, seed=1, device=0, coeff_mode=mode)
os.environ.pop("DFAMD_HANDOFF_BATCH")
res = {v: [] for v in hs}
for f in hs.values():
    for _ in range(32):
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
st = {v: f.rng_state() for v, f in hs.items()}
print(json.dumps({"config": cfg, "mode": mode, "ms_per_call_median": {v: round(statistics.median(x), 4) for v, x in res.items()},
                  "ms_per_call_min": {v: round(min(x), 4) for v, x in res.items()},
                  "same_stream_state": len(set(st.values())) == 1}))
