#!/usr/bin/env python3
"""Wall time per filter(dt) call with profiling OFF (the HIP-graph path needs it off), graph 0 vs 1
on one handle, interleaved rounds; small planes are bound by the host's launch rate.

    python3 tools/graph_ab.py [--config c1] [--mode packed] [--calls 200] [--rounds 7]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
import dfamd  # noqa: E402

CFG = {"c1": (128, 128, 8, 8), "c2": (512, 512, 4, 32), "native": None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1")
    ap.add_argument("--mode", default="packed")
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    if CFG[a.config] is None:
        f = dfamd.DigitalFilter(seed=1, device=0, coeff_mode=a.mode)
    else:
        Ny, Nz, lo, hi = CFG[a.config]
        f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=1, device=0,
                                coeff_mode=a.mode)
    rec = {0: [], 1: []}
    for _ in range(a.rounds):
        for gr in (0, 1):
            f.set_tuning("graph", gr)
            for _ in range(5):
                f.filter(1e-8)
            f.sync()
            t0 = time.perf_counter()
            for _ in range(a.calls):
                f.filter(1e-8)
            f.sync()
            rec[gr].append((time.perf_counter() - t0) * 1e6 / a.calls)
    print(json.dumps({"config": a.config, "mode": a.mode,
                      "us_per_call": {f"graph{g}": round(statistics.median(v), 2) for g, v in rec.items()}}))


if __name__ == "__main__":
    main()
