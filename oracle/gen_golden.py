#!/usr/bin/env python3
"""Generate tests/golden/ from the REFERENCE itself (oracle/_ref/, built by
`make -C oracle/ref` from the unmodified sources under /root/reference).

Run in the build container only (it needs the reference build):
    make -C oracle/ref && make -C oracle && python3 oracle/gen_golden.py

Every fixture is data: inputs (seeds, plane specs, dt) and the outputs the
reference produced for them. The oracle restatement (df_oracle.c) is then
required to reproduce these bit for bit (tests/test_oracle_golden.py).
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = os.path.join(HERE, "_ref")
HARN = os.path.join(REF, "ref_harness")
RUN_ROOT = os.path.join(REF, "run_root")
OUT = os.path.join(ROOT, "tests", "golden")
FIELDS = ("u", "v", "w", "T", "rho")
ROWS = ("R11", "R21", "R22", "R33", "Us", "Ts", "rhos", "Ms")
KAT = "/root/reference/digital-filtering-c++/pcg-cpp/test-high/expected/check-pcg32.out"

sys.path.insert(0, HERE)
import oracle as O  # noqa: E402  (only to record the derived stream start state)


def run(*args):
    subprocess.run([HARN, *map(str, args)], check=True, stdout=subprocess.DEVNULL)


def stats(a):
    return np.array([a.sum(), (a * a).sum(), np.abs(a).max()])


def load_case(d, Ny, Nz, nsteps):
    meta = json.load(open(os.path.join(d, "meta.json")))
    rows = {r: np.fromfile(os.path.join(d, r + ".bin")) for r in ROWS}
    Ns = {}
    for c in "uvw":
        for dn in "yz":
            a = np.fromfile(os.path.join(d, f"N{dn}s_{c}.bin"), dtype=np.int32).reshape(meta["Ny"], meta["Nz"])
            assert (a == a[:, :1]).all(), "half-width is not uniform along a row"
            Ns[f"N{dn}_{c}"] = a[:, 0].copy()
    steps = []
    for s in range(nsteps + 1):
        steps.append({k: np.fromfile(os.path.join(d, f"step{s}_{k}.bin")).reshape(meta["Ny"], meta["Nz"])
                      for k in FIELDS})
    return meta, rows, Ns, steps


def kat():
    lines = [l.rstrip("\r\n") for l in open(KAT)]
    r1 = lines.index("Round 1:")
    first = [int(x, 16) for x in lines[r1 + 1].split(":")[1].split()]
    again = [int(x, 16) for x in lines[r1 + 2].split(":")[1].split()]
    coins = lines[r1 + 3].split(":")[1].strip()
    json.dump({"source": "pcg-cpp/test-high/expected/check-pcg32.out (reference's own KAT)",
               "seed": 42, "stream": 54, "round1_32bit": first, "round1_again": again,
               "round1_coins": coins}, open(os.path.join(OUT, "pcg32_kat.json"), "w"), indent=1)


def rng_fixture(seed, n=4096):
    with tempfile.TemporaryDirectory() as d:
        run("rng", seed, n, d)
        u = np.fromfile(os.path.join(d, "u32.bin"), dtype=np.uint32)
        g = np.fromfile(os.path.join(d, "normals.bin"))
    np.savez_compressed(os.path.join(OUT, f"rng_s{seed}.npz"), seed=seed, u32=u, normals=g)


def native_fixture(seed=42, dt=1e-8, nsteps=2, sample_rows=(1, 100, 300, 509)):
    with tempfile.TemporaryDirectory() as d:
        run("native", RUN_ROOT, seed, dt, nsteps, d)
        meta, rows, Ns, steps = load_case(d, 0, 0, nsteps)
    arr = {"seed": seed, "dt": dt, "nsteps": nsteps, "sample_rows": np.array(sample_rows)}
    arr.update({f"row_{k}": v for k, v in rows.items()})
    arr.update(Ns)
    for s, st in enumerate(steps):
        for k in FIELDS:
            arr[f"s{s}_{k}_stats"] = stats(st[k])
            arr[f"s{s}_{k}_rows"] = st[k][list(sample_rows)]
    np.savez_compressed(os.path.join(OUT, f"native_s{seed}.npz"), **arr)
    json.dump(meta, open(os.path.join(OUT, f"native_s{seed}.json"), "w"), indent=1)


def sha256(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def synth_fixture(name, seed, Ny, Nz, Nmin, Nmax, dt, nsteps, dt2=None, nsteps2=0, full_steps=(),
                  sample_rows=None, csv_head=0, hashes=False):
    with tempfile.TemporaryDirectory() as d:
        extra = [dt2, nsteps2] if nsteps2 else []
        run("synth", RUN_ROOT, seed, Ny, Nz, Nmin, Nmax, dt, nsteps, d, *extra)
        meta, rows, Ns, steps = load_case(d, Ny, Nz, nsteps + nsteps2)
        if csv_head:
            with open(os.path.join(RUN_ROOT, "files", "cpp_vel_fluc.csv")) as f:
                head = [next(f) for _ in range(csv_head)]
            open(os.path.join(OUT, f"{name}_csv_head.txt"), "w").writelines(head)
    # The reference runs its native constructor first (one process-wide static
    # stream, df.cpp:334-335); record where the synthetic plane's stream starts.
    rng = O.Rng(seed=seed)
    O.Filter(rng=rng)
    st, flag, saved = rng.state
    sample_rows = sample_rows or (0, 1, Ny // 4, Ny // 2, Ny - 1)
    arr = {"seed": seed, "Ny": Ny, "Nz": Nz, "N_min": Nmin, "N_max": Nmax, "dt": dt, "nsteps": nsteps,
           "dt2": dt2 if dt2 is not None else 0.0, "nsteps2": nsteps2,
           "start_state": np.uint64(st), "start_saved_flag": flag, "start_saved": saved,
           "sample_rows": np.array(sample_rows), "full_steps": np.array(full_steps, dtype=np.int64)}
    arr.update({f"row_{k}": v for k, v in rows.items()})
    arr.update(Ns)
    for s, stp in enumerate(steps):
        for k in FIELDS:
            arr[f"s{s}_{k}_stats"] = stats(stp[k])
            arr[f"s{s}_{k}_rows"] = stp[k][list(sample_rows)]
            if s in full_steps:
                arr[f"s{s}_{k}"] = stp[k]
            if hashes:  # the whole field, bit for bit, in 64 hex digits (planes too large to keep)
                arr[f"s{s}_{k}_sha256"] = np.array(sha256(stp[k]))
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arr)
    json.dump(meta, open(os.path.join(OUT, f"{name}.json"), "w"), indent=1)


def grid_fixture(name, seed, Ny, Nz, dt, nsteps, full_steps=(), **grid_kw):
    """Real-grid plane: caller vertices with per-cell dy, dz, yc, so the
    half-widths vary per cell; setup, coefficients and the hot path are the reference's."""
    gy, gz = O.warped_grid(Ny, Nz, **grid_kw)
    with tempfile.TemporaryDirectory() as d:
        vf = os.path.join(d, "vert.bin")
        with open(vf, "wb") as f:
            np.array([Ny, Nz], dtype=np.int32).tofile(f)
            gy.tofile(f)
            gz.tofile(f)
        run("grid", RUN_ROOT, seed, vf, dt, nsteps, d)
        meta = json.load(open(os.path.join(d, "meta.json")))
        ny, nz = meta["Ny"], meta["Nz"]
        rows = {r: np.fromfile(os.path.join(d, r + ".bin")) for r in ROWS}
        Ns = {f"N{dn}_{c}": np.fromfile(os.path.join(d, f"N{dn}s_{c}.bin"), dtype=np.int32).reshape(ny, nz)
              for c in "uvw" for dn in "yz"}
        steps = [{k: np.fromfile(os.path.join(d, f"step{s}_{k}.bin")).reshape(ny, nz) for k in FIELDS}
                 for s in range(nsteps + 1)]
    assert any((Ns[k] != Ns[k][:, :1]).any() for k in Ns), "grid does not vary the half-width per cell"
    rng = O.Rng(seed=seed)
    O.Filter(rng=rng)
    st, flag, saved = rng.state
    arr = {"seed": seed, "Ny_in": Ny, "Nz_in": Nz, "Ny": ny, "Nz": nz, "dt": dt, "nsteps": nsteps,
           "grid_y": gy, "grid_z": gz, "start_state": np.uint64(st), "start_saved_flag": flag,
           "start_saved": saved, "full_steps": np.array(full_steps, dtype=np.int64)}
    arr.update({f"row_{k}": v for k, v in rows.items()})
    arr.update(Ns)
    for s, stp in enumerate(steps):
        for k in FIELDS:
            arr[f"s{s}_{k}_stats"] = stats(stp[k])
            if s in full_steps:
                arr[f"s{s}_{k}"] = stp[k]
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arr)
    json.dump(meta, open(os.path.join(OUT, f"{name}.json"), "w"), indent=1)


def rms_fixture(name, seed, synth=None, sample_rows=None, csv_head=12):
    """The reference driver's own path: DIGITAL_FILTER df(config); df.get_rms() (cpp-main.cpp:12-17)."""
    with tempfile.TemporaryDirectory() as d:
        run("rms", RUN_ROOT, seed, d, *(synth or ()))
        meta = json.load(open(os.path.join(d, "meta.json")))
        Ny, Nz = meta["Ny"], meta["Nz"]
        rms = {k: np.fromfile(os.path.join(d, f"rms_{k}.bin")).reshape(Ny, Nz) for k in FIELDS}
        with open(os.path.join(RUN_ROOT, "files", "cpp_vel_fluc_rms.csv")) as f:
            head = [next(f) for _ in range(csv_head)]
    open(os.path.join(OUT, f"{name}_csv_head.txt"), "w").writelines(head)
    sample_rows = sample_rows or (1, Ny // 4, Ny // 2, Ny - 1)
    arr = {"seed": seed, "Ny": Ny, "Nz": Nz, "rms_counter": meta["rms_counter"],
           "synth": np.array(synth or (), dtype=np.int64), "sample_rows": np.array(sample_rows)}
    for k in FIELDS:
        arr[f"rms_{k}_stats"] = stats(rms[k])
        arr[f"rms_{k}_rows"] = rms[k][list(sample_rows)]
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arr)


def writers_fixture(name, seed=42, dt=1e-8, nsteps=2, every=997):
    """The reference's file writers on its native grid (f4): the per-call CSV of filter()
    (df.cpp:466-467, 764-803), write_tecplot (712-762) and plot_RST_lerp (677-706). The CSV and
    Tecplot files (~20 MB each) are kept as header + line count + every `every`-th line + the
    sha256 of the coordinate text; myRST.csv / duanRST.csv (a few hundred lines) whole."""
    import hashlib
    files = os.path.join(RUN_ROOT, "files")
    with tempfile.TemporaryDirectory() as d:
        run("writers", RUN_ROOT, seed, dt, nsteps, d)
        tec = open(os.path.join(d, "tecplot.dat")).read().splitlines()
    csv = open(os.path.join(files, "cpp_vel_fluc.csv")).read().splitlines()
    meta = {"seed": seed, "dt": dt, "nsteps": nsteps, "every": every}
    # Tecplot BLOCK: 3 header lines, (Ny+1)(Nz+1) z then y vertex values, then u, v, w per cell
    nv = 511 * 401
    coords = tec[3:3 + 2 * nv]
    meta["tecplot"] = {"header": tec[:3], "n_lines": len(tec),
                       "coord_sha256": hashlib.sha256("\n".join(coords).encode()).hexdigest(),
                       "sample": {str(i): tec[i] for i in range(3, len(tec), every)}}
    cz = [",".join(l.split(",")[:2]) for l in csv[1:]]
    meta["csv"] = {"header": csv[0], "n_lines": len(csv),
                   "coord_sha256": hashlib.sha256("\n".join(cz).encode()).hexdigest(),
                   "sample": {str(i): csv[i] for i in range(1, len(csv), every)}}
    json.dump(meta, open(os.path.join(OUT, f"{name}.json"), "w"), indent=0)
    for f in ("myRST.csv", "duanRST.csv"):
        open(os.path.join(OUT, f"{name}_{f}"), "w").write(open(os.path.join(files, f)).read())


def main():
    if not os.path.exists(HARN):
        sys.exit("reference not built: make -C oracle/ref")
    os.makedirs(OUT, exist_ok=True)
    if len(sys.argv) > 1:  # regenerate named fixtures only, e.g. `gen_golden.py writers`
        for name in sys.argv[1:]:
            {"writers": lambda: writers_fixture("writers_native_s42"), "c2": c2_fixture}[name]()
        manifest()
        return
    kat()
    rng_fixture(42)
    rng_fixture(1234)
    native_fixture()
    # c1: 128x128, constant N = 8 (BASELINE configs[0]); 3 x filter(1e-8) then filter(1e-5)
    synth_fixture("c1_s42", 42, 128, 128, 8, 8, 1e-8, 3, dt2=1e-5, nsteps2=1, full_steps=(3,),
                  csv_head=12)
    # small ramp-rule plane (SURVEY §8d rule, N in [4,16]) on another seed
    synth_fixture("ramp256_s1234", 1234, 256, 256, 4, 16, 1e-8, 2)
    # ragged plane: odd sizes, Nz smaller than the largest half-width
    synth_fixture("ragged_s7", 7, 37, 5, 2, 10, 1e-8, 2, full_steps=(0, 2), sample_rows=(0, 18, 36))
    # real-grid plane: vertices vary along z, half-widths vary per cell; 2 strips, ragged
    grid_fixture("grid_s3", 3, 60, 200, 1e-8, 2, full_steps=(0, 2))
    # the reference driver's get_rms() (500 steps at dt = 1e-5) on its native grid
    rms_fixture("rms_native_s42", 42)
    # the reference's file writers on its native grid: per-call CSV, write_tecplot, plot_RST_lerp
    writers_fixture("writers_native_s42")
    c2_fixture()
    manifest()


def c2_fixture():
    # c2 (BASELINE configs[1]): 512 x 512, N 4-32 by the SURVEY 8d rule, step 0 + 2 x filter(1e-8): sampled rows,
    # stats and the sha256 of every whole field at every step (round 5)
    synth_fixture("c2_s42", 42, 512, 512, 4, 32, 1e-8, 2, sample_rows=(0, 1, 100, 128, 256, 511), hashes=True)


def manifest():
    manifest = {
        "generator": "oracle/gen_golden.py",
        "reference": "connorswitala/digital-filtering @ /root/reference (df.cpp compiled unmodified, "
                     "g++ -std=c++17 -O2, -include oracle/ref/ref_shim.hpp)",
        "compiler": subprocess.run(["g++", "--version"], capture_output=True, text=True).stdout.splitlines()[0],
        "files": sorted(os.listdir(OUT)),
    }
    json.dump(manifest, open(os.path.join(OUT, "MANIFEST.json"), "w"), indent=1)
    print("wrote", OUT)
    return manifest


if __name__ == "__main__":
    main()
