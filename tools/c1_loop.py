#!/usr/bin/env python3
"""c1 (128 x 128, N = 8) in a loop, for a kernel trace of a launch-bound plane:
    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 tools/c1_loop.py [calls] [mode]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "digital-filtering_amd"))
import torch  # noqa: E402,F401
import dfamd  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
mode = sys.argv[2] if len(sys.argv) > 2 else "packed"
f = dfamd.DigitalFilter(plane="synthetic", Ny=128, Nz=128, N_min=8, N_max=8, seed=1, device=0, coeff_mode=mode)
for _ in range(calls):
    f.filter(1e-8)
f.sync()
