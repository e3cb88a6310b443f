#!/usr/bin/env python3
"""In-process A/B timing of library variants on one GPU (guide §5.4 rule 24).

    python3 tools/ab.py --a "DFAMD_RNG_OVERLAP=1" --b "DFAMD_RNG_OVERLAP=0" [--config c3] [--mode table]

Each variant is a separate handle created with its env knobs set; the handles
run interleaved rounds of K calls and the per-phase hipEvent times are reported
as median over rounds.

    python3 tools/ab.py --tune-a rows_per_wave=4 --tune-b rows_per_wave=2,yunroll=4

--tune-* variants run on ONE handle (df_set_tuning between rounds), so both see
the same allocations: separate handles differ by up to ~4% from page placement.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
if "--torch" in sys.argv:  # bind libdfamd to torch's HIP runtime first, as bench.py does
    sys.argv.remove("--torch")
    import torch  # noqa: F401
    torch.cuda.set_device(0)
import dfamd  # noqa: E402

CFG = {"c1": (128, 128, 8, 8), "c2": (512, 512, 4, 32), "c3": (2048, 2048, 4, 64), "c5": (4096, 4096, 4, 64),
       "native": None}  # the reference's own grid and profiles (510 x 400)


def make(envspec, cfg, mode, rpw):
    saved = {}
    for kv in filter(None, envspec.replace(":", ",").split(",")):
        k, v = kv.split("=")
        saved[k] = os.environ.get(k)
        os.environ[k] = v
    if CFG[cfg] is None:
        f = dfamd.DigitalFilter(plane=cfg, seed=1, device=0, coeff_mode=mode, rows_per_wave=rpw)
    else:
        Ny, Nz, a, b = CFG[cfg]
        f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=a, N_max=b, seed=1, device=0,
                                coeff_mode=mode, rows_per_wave=rpw)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default="")
    ap.add_argument("--b", default="")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--mode", default="packed")
    ap.add_argument("--rpw-a", type=int, default=0)
    ap.add_argument("--rpw-b", type=int, default=0)
    ap.add_argument("--tune-a", default=None)
    ap.add_argument("--tune-b", default=None)
    ap.add_argument("--rounds", type=int, default=7)
    # 60: pipelines that run ahead (noise epochs, the y-pass ahead) hold several calls of work past a window's
    # last call; 10-call windows timed the first setting of each round ~40% slower (profiles/r5/m)
    ap.add_argument("--calls", type=int, default=60)
    ap.add_argument("--events", type=int, default=1, help="0: wall time only (no per-call phase events)")
    ap.add_argument("--switch-calls", type=int, default=1,
                    help="untimed calls after a --tune switch (a pipeline form takes effect an epoch later)")
    a = ap.parse_args()
    tune = None
    if a.tune_a is not None or a.tune_b is not None:
        one = make(a.a, a.config, a.mode, a.rpw_a)
        hs = {"A": one, "B": one}
        tune = {k: [(kv.split("=")[0], int(kv.split("=")[1])) for kv in filter(None, (v or "").replace(":", ",").split(","))]
                for k, v in (("A", a.tune_a), ("B", a.tune_b))}
    else:
        hs = {"A": make(a.a, a.config, a.mode, a.rpw_a), "B": make(a.b, a.config, a.mode, a.rpw_b)}
    rec = {k: {p: [] for p in ("rng_ms", "ypass_ms", "zpass_ms", "total_ms", "wall_ms")} for k in hs}
    for f in hs.values():
        for _ in range(3):
            f.filter(1e-8)
        f.sync()
    for _ in range(a.rounds):
        for k, f in hs.items():
            if tune is not None:
                for key, val in tune[k]:
                    f.set_tuning(key, val)
                for _ in range(a.switch_calls):
                    f.filter(1e-8)  # calls right after a switch are not timed
            f.set_profiling(bool(a.events))
            f.sync()
            t0 = time.perf_counter()
            for _ in range(a.calls):
                f.filter(1e-8)
            f.sync()
            wall = (time.perf_counter() - t0) * 1e3 / a.calls
            p = f.profile() if a.events else {"calls": 1, "rng_ms": 0, "ypass_ms": 0, "zpass_ms": 0, "total_ms": 0}
            f.set_profiling(False)
            p["wall_ms"] = wall * p["calls"]
            for ph in rec[k]:
                rec[k][ph].append(p[ph] / p["calls"])
    out = {"A": a.tune_a if tune else a.a, "B": a.tune_b if tune else a.b, "config": a.config, "mode": a.mode}
    for k in hs:
        out[k + "_median_ms"] = {ph: round(statistics.median(v), 4) for ph, v in rec[k].items()}
        out[k + "_min_ms"] = {ph: round(min(v), 4) for ph, v in rec[k].items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
