#!/usr/bin/env python3
"""Sweep of df_set_tuning settings on ONE handle (same allocations), interleaved rounds.

    python3 tools/win_sweep.py [--config c3] [--mode packed] [--rounds 5] [--calls 10] \
        --set "zwin_T=4096,zwin_W=256" --set "ywin_T=4096,ywin_W=256" ...

Every --set is applied on top of the knobs' reset values given by --base (default: the
write-window knobs off). Prints one JSON line: per setting, median per-phase ms per call.
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

CFG = {"c2": (512, 512, 4, 32), "c3": (2048, 2048, 4, 64), "c5": (4096, 4096, 4, 64)}


def parse_kv(s):
    return [(kv.split("=")[0], int(kv.split("=")[1])) for kv in filter(None, s.split(","))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--mode", default="packed")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--base", default="ywin_T=0,ywin_W=0,zwin_T=0,zwin_W=0")
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    Ny, Nz, lo, hi = CFG[a.config]
    f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=1, device=0,
                            coeff_mode=a.mode)
    settings = ["base"] + a.set
    rec = {s: {p: [] for p in ("rng_ms", "ypass_ms", "zpass_ms", "total_ms", "wall_ms")} for s in settings}
    for _ in range(3):
        f.filter(1e-8)
    f.sync()
    for _ in range(a.rounds):
        for s in settings:
            for k, v in parse_kv(a.base) + ([] if s == "base" else parse_kv(s)):
                f.set_tuning(k, v)
            f.filter(1e-8)
            f.set_profiling(True)
            f.sync()
            t0 = time.perf_counter()
            for _ in range(a.calls):
                f.filter(1e-8)
            f.sync()
            wall = (time.perf_counter() - t0) * 1e3 / a.calls
            p = f.profile()
            f.set_profiling(False)
            p["wall_ms"] = wall * p["calls"]
            for ph in rec[s]:
                rec[s][ph].append(p[ph] / p["calls"])
        print(f"round done", file=sys.stderr, flush=True)
    out = {"config": a.config, "mode": a.mode, "base": a.base,
           "median_ms": {s: {ph: round(statistics.median(v), 4) for ph, v in rec[s].items()} for s in settings}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
