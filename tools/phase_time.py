#!/usr/bin/env python3
"""Per-phase device time of filter(dt) for one handle (timing experiments; not a test).

    python3 tools/phase_time.py --config c3|native|...  (DFAMD_LIB=<another build of libdfamd.so> to time that one)

Prints one JSON line: median over rounds of the hipEvent phase times (ms per call).
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
import torch  # noqa: E402,F401  (one HIP runtime per process, as bench.py)
import dfamd  # noqa: E402

CFG = {"c1": (128, 128, 8, 8), "c2": (512, 512, 4, 32), "c3": (2048, 2048, 4, 64), "c5": (4096, 4096, 4, 64),
       "u64": (2048, 2048, 64, 64), "u16": (2048, 2048, 16, 16), "c3big": (4096, 2048, 4, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--mode", default="packed")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--tune", default="")
    a = ap.parse_args()
    if a.config == "native":  # the reference's own 510 x 400 grid
        f = dfamd.DigitalFilter(plane="native", seed=1, device=0, coeff_mode=a.mode)
    else:
        Ny, Nz, lo, hi = CFG[a.config]
        f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=1, device=0,
                                coeff_mode=a.mode)
    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        f.set_tuning(k, int(v))
    for _ in range(3):
        f.filter(1e-8)
    f.sync()
    rec = {p: [] for p in ("rng_ms", "ypass_ms", "zpass_ms", "total_ms")}
    for _ in range(a.rounds):
        f.set_profiling(True)
        for _ in range(a.calls):
            f.filter(1e-8)
        f.sync()
        p = f.profile()
        f.set_profiling(False)
        for k in rec:
            rec[k].append(p[k] / p["calls"])
    out = {"lib": os.path.basename(dfamd.LIB_PATH), "config": a.config, "mode": a.mode, "tune": a.tune}
    out.update({k: round(statistics.median(v), 4) for k, v in rec.items()})
    out["ypass_GBps"] = round(f.algorithmic_bytes(0) / out["ypass_ms"] / 1e6, 1)
    out["zpass_GBps"] = round(f.algorithmic_bytes(1) / out["zpass_ms"] / 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
