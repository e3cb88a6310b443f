import sys, time, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "digital-filtering_amd"))
import torch, dfamd
for spec in [(128, 128, 8, 8), (512, 512, 4, 32)]:
    f = dfamd.DigitalFilter(plane="synthetic", Ny=spec[0], Nz=spec[1], N_min=spec[2], N_max=spec[3], seed=1, device=0)
    for _ in range(20): f.filter(1e-8)
    f.sync()
    t0 = time.perf_counter()
    for _ in range(500): f.filter(1e-8)
    f.sync()
    t1 = time.perf_counter()
    for _ in range(200):
        f.filter(1e-8); f.sync()
    t2 = time.perf_counter()
    f.set_profiling(True)
    for _ in range(100): f.filter(1e-8)
    f.sync(); p = f.profile()
    print(spec, "async us/call %.1f" % ((t1 - t0) / 500 * 1e6), "sync us/call %.1f" % ((t2 - t1) / 200 * 1e6),
          {k: round(p[k] / p["calls"] * 1e3, 1) for k in ("rng_ms", "ypass_ms", "zpass_ms", "total_ms")})
