#!/usr/bin/env python3
"""One rank of an N-way z-strip split on one GPU (DFAMD_SOLO_STRIP timing mode; fields meaningless), for
rocprofv3 per-kernel breakdowns of the per-rank work:
    rocprofv3 --kernel-trace --stats -- python3 tools/solo_rank.py --N 8 --rank 4 --mode table --config c4 \
        --tune gen_dense=2"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
os.environ["DFAMD_SOLO_STRIP"] = "1"
p = argparse.ArgumentParser()
p.add_argument("--N", type=int, default=8)
p.add_argument("--rank", type=int, default=4)
p.add_argument("--mode", default="table", choices=["packed", "table"])
p.add_argument("--config", default="c4", choices=["c4", "c5", "weak"])
p.add_argument("--calls", type=int, default=20)
p.add_argument("--replicate", type=int, default=None)
p.add_argument("--tune", default="", help="k=v,... df_set_tuning after create")
a = p.parse_args()
import dfamd  # noqa: E402

Ny, Nz = {"c4": (2048, 8192), "c5": (4096, 4096), "weak": (2048, 2048 * a.N)}[a.config]
f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=4, N_max=64, seed=1, device=0, rank=a.rank,
                        world=a.N, coeff_mode=a.mode)
if a.replicate is not None:
    f.set_tuning("rng_replicate", a.replicate)
for kv in filter(None, a.tune.split(":")):
    f.set_tuning(kv.split("=")[0], int(kv.split("=")[1]))
for _ in range(a.calls):
    f.filter(1e-8)
f.sync()
