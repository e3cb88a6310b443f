"""Debug: one ghost-column strip group in isolation, progress printed after every step."""
import faulthandler
import os
import sys

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import dfamd  # noqa: E402
import oracle as O  # noqa: E402

world, Ny, Nz, lo, hi = (int(x) for x in sys.argv[1:6])
tuning = dict(kv.split("=") for kv in sys.argv[6:])
tuning = {k: int(v) for k, v in tuning.items()}
print("create", flush=True)
hs = dfamd.create_group(world, plane="synthetic", Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=19, device=0,
                        coeff_mode="table")
for f in hs:
    for k, v in dict(halo_ghost=1, **tuning).items():
        print("set", f.z0, k, v, flush=True)
        f.set_tuning(k, v)
        f.sync()
o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=19)
for i in range(3):
    print("call", i, flush=True)
    o.filter(1e-8)
    dfamd.filter_group(hs, 1e-8)
    for f in hs:
        f.sync()
    ok = all(np.array_equal(np.concatenate([h.field(k) for h in hs], axis=1), o.field(k)) for k in ("u", "v", "w"))
    print("equal", ok, flush=True)
