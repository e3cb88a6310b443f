#!/usr/bin/env python3
"""One rank of an N-way z-strip split on one GPU (DFAMD_SOLO_STRIP timing mode; fields
meaningless). For rocprofv3 per-kernel breakdowns of the per-rank work:
    rocprofv3 --kernel-trace --stats -- python3 tools/solo_rank.py N rank [packed|table] [calls]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
os.environ["DFAMD_SOLO_STRIP"] = "1"
import torch  # noqa: E402,F401
import dfamd  # noqa: E402

N, rank = int(sys.argv[1]), int(sys.argv[2])
mode = sys.argv[3] if len(sys.argv) > 3 else "packed"
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 10
f = dfamd.DigitalFilter(plane="synthetic", Ny=2048, Nz=2048 * N, N_min=4, N_max=64, seed=1, device=0,
                        rank=rank, world=N, coeff_mode=mode)
for _ in range(calls):
    f.filter(1e-8)
f.sync()
