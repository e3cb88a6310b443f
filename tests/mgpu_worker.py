"""One rank of a multi-process z-strip run (tests/test_gpu_multi.py starts one per GPU).

Creates its strip with the shared RCCL id (df_create: ncclCommInitRank, step 0 with the
halo send/recv to its neighbours), runs `calls` filter(dt) calls, then runs the whole plane
unsplit on its own GPU and compares its strip with it bit for bit. Prints one JSON line.

    python tests/mgpu_worker.py '<json spec>'
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "digital-filtering_amd"))
import dfamd  # noqa: E402


def main():
    spec = json.loads(sys.argv[1])
    rank, world = spec["rank"], spec["world"]
    plane = dict(plane="synthetic", Ny=spec["Ny"], Nz=spec["Nz"], N_min=spec["N_min"], N_max=spec["N_max"],
                 seed=spec["seed"], coeff_mode=spec["mode"], device=spec.get("device", rank))
    h = dfamd.DigitalFilter(rank=rank, world=world, comm_id=bytes.fromhex(spec["comm_id"]), **plane)
    if "replicate" in spec:  # 1: every rank counts the whole stream; 0: split counting + the counts all-gather
        h.set_tuning("rng_replicate", int(spec["replicate"]))
    if "halo_overlap" in spec:  # 0: pack, send/recv, unpack and the whole z-pass as one chain on the stream
        h.set_tuning("halo_overlap", int(spec["halo_overlap"]))
    for k, v in spec.get("tuning", {}).items():  # e.g. gen_dense 2: run generation + fused exchange
        h.set_tuning(k, int(v))
    for dt in spec["dts"]:
        h.filter(dt)
    h.sync()
    comm = h.comm_info()
    ref = dfamd.DigitalFilter(**dict(plane, coeff_mode=spec.get("ref_mode", "table")))
    for dt in spec["dts"]:
        ref.filter(dt)
    bad = {}
    for k in ("u", "v", "w", "T", "rho", "filt_old_u", "filt_old_v", "filt_old_w"):
        a = h.field(k)
        b = np.ascontiguousarray(ref.field(k)[:, h.z0:h.z1])
        n = int(np.count_nonzero(a.view(np.uint64) != b.view(np.uint64)))
        if n:
            bad[k] = n
    out = {"rank": rank, "columns": [h.z0, h.z1], "mismatch": bad,
           "rng_equal": h.rng_state() == ref.rng_state(), "comm": comm}
    ref.close()
    h.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
