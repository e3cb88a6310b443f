#!/usr/bin/env python3
"""Launch-shape sweep on ONE handle (df_set_tuning between settings, so every setting sees
the same allocations): median hipEvent phase times per setting, interleaved over rounds.

    python3 tools/tune_sweep.py --plane native --mode packed \\
        "rows_per_wave=2" "rows_per_wave=1,yunroll=4" ...
Prints one JSON line per setting."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "digital-filtering_amd"))
import torch  # noqa: E402,F401
import dfamd  # noqa: E402

SYN = {"c1": (128, 128, 8, 8), "c2": (512, 512, 4, 32), "c3": (2048, 2048, 4, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plane", default="native")
    ap.add_argument("--mode", default="packed")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--comm", action="store_true",
                    help="one-rank RCCL handle (world 1 with a communicator): halo_loopback/halo_overlap apply")
    ap.add_argument("settings", nargs="+")
    a = ap.parse_args()
    if a.plane in SYN:
        Ny, Nz, lo, hi = SYN[a.plane]
        extra = dict(rank=0, world=1, comm_id=dfamd.comm_unique_id()) if a.comm else {}
        f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=1, device=0,
                                coeff_mode=a.mode, **extra)
    else:
        f = dfamd.DigitalFilter(plane=a.plane, seed=1, device=0, coeff_mode=a.mode)
    sets = [[(kv.split("=")[0], int(kv.split("=")[1])) for kv in s.split(",") if kv] for s in a.settings]
    rec = [{p: [] for p in ("rng_ms", "ypass_ms", "zpass_ms", "total_ms")} for _ in sets]
    for _ in range(a.rounds):
        for i, st in enumerate(sets):
            for k, v in st:
                f.set_tuning(k, v)
            for _ in range(3):
                f.filter(1e-8)
            f.sync()
            f.set_profiling(True)
            for _ in range(a.calls):
                f.filter(1e-8)
            f.sync()
            p = f.profile()
            f.set_profiling(False)
            for k in rec[i]:
                rec[i][k].append(p[k] / p["calls"] * 1e3)
    for s, r in zip(a.settings, rec):
        print(json.dumps({"plane": a.plane, "mode": a.mode, "setting": s,
                          "median_us": {k: round(statistics.median(v), 1) for k, v in r.items()}}), flush=True)


if __name__ == "__main__":
    main()
