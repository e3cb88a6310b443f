#!/usr/bin/env python3
"""Benchmark of DIGITAL_FILTER::filter(dt) on MI355X (BASELINE.json metric).

One step = one filter(dt) call (reference df.cpp:449-468) over the whole plane:
device RNG in the reference's stream order, y- and z-convolutions streaming the
offset-packed coefficients, correlation, RST scaling, SRA T'/rho'.

Workload (N=1): BASELINE configs[2] / SURVEY c3 — 2048 x 2048 plane, half-width
rule N in [4, 64], dt = 1e-8, synthetic rows from files/RST.dat + line.dat.
N>1 (weak scaling): one 2048 x 2048 z-strip per GPU of a 2048 x (2048 N) plane,
one RCCL halo exchange per call (N=4 is SURVEY c4's 2048 x 8192 plane).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--coeff-mode packed|table]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "digital-filtering_amd")
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (Ny, Nz per GPU, N_min, N_max, description)
    "c1": (128, 128, 8, 8, "c1: 128x128 plane, constant half-width N=8"),
    "c2": (512, 512, 4, 32, "c2: 512x512 plane, half-width 4-32"),
    "c3": (2048, 2048, 4, 64, "c3: 2048x2048 plane per GPU, half-width 4-64 (HBM roofline point)"),
    "c5": (4096, 4096, 4, 64, "c5: 4096x4096 plane per GPU, half-width 4-64"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--coeff-mode", default="packed", choices=["packed", "table"])
    p.add_argument("--rows-per-wave", type=int, default=0)  # 0 = library default per mode
    p.add_argument("--dt", type=float, default=1e-8)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    p.add_argument("--cpu-cols", type=int, default=512,
                   help="columns of the CPU sample (same rows and half-width rule as the GPU plane)")
    p.add_argument("--cpu-calls", type=int, default=16)  # ~13 s of reference CPU work (0.8 s per call)
    p.add_argument("--pmc-file", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--other-configs", default="",
                   help="comma list of further single-GPU configs timed after the main one (N=1 only), e.g. c2; "
                        "off by default so that rocprofv3 averages of the default command cover c3 launches only")
    p.add_argument("--alt-modes", default="auto", choices=["auto", "off"],
                   help="also time the other coefficient mode (N=1 only) and report it under alt_modes")
    return p.parse_args()


def cpu_baseline(args, Ny, N_min, N_max):
    """Reference CPU path on this host: df.cpp built from the reference sources
    (oracle/_ref/ref_harness, g++ -O2, 1 thread), else the oracle restatement."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    run_root = os.path.join(ROOT, "oracle", "_ref", "run_root")
    nz = args.cpu_cols
    sample = (f"{Ny}x{nz} (the GPU plane's {Ny} rows and N {N_min}-{N_max} rule, {nz} columns), "
              f"{args.cpu_calls} filter(dt) calls after construction")
    if os.path.exists(exe) and os.path.isdir(run_root):
        out = subprocess.run([exe, "time", run_root, str(args.seed), str(Ny), str(nz), str(N_min), str(N_max),
                              str(args.dt), str(args.cpu_calls)], capture_output=True, text=True, check=True)
        rec = json.loads(out.stdout.strip().splitlines()[-1])
        return {"value": Ny * nz / rec["mean_s"], "unit": "cells/s", "cores": 1, "kind": "reference",
                "sample": sample, "s_per_call": rec["mean_s"],
                "stage_s": {k: rec[k] for k in ("noise_s", "sweeps_s", "correlate_s", "rst_s", "sra_s")}}
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=Ny, Nz=nz, N_min=N_min, N_max=N_max, seed=args.seed)
    t0 = time.perf_counter()
    for _ in range(args.cpu_calls):
        o.filter(args.dt)
    dt = (time.perf_counter() - t0) / args.cpu_calls
    return {"value": Ny * nz / dt, "unit": "cells/s", "cores": 1, "kind": "port", "sample": sample,
            "s_per_call": dt}


PAR_SCRIPT = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
import oracle as O
Ny, Nz, lo, hi, seed, dt, calls = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), \
    int(sys.argv[6]), float(sys.argv[7]), int(sys.argv[8])
o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=Ny, Nz=Nz, N_min=lo, N_max=hi, seed=seed)
o.filter(dt)
t0 = time.perf_counter()
for _ in range(calls):
    o.filter(dt)
print(json.dumps({"s_per_call": (time.perf_counter() - t0) / calls}))
"""


def cpu_baseline_parallel(args, Ny, N_min, N_max):
    """The oracle restatement built with OpenMP over the sweep rows (oracle/liboracle_omp.so; the
    RNG stays serial as in the reference) on this host's cores: a multi-core CPU figure beside the
    single-threaded reference. Not the reference; same bits (tests/test_oracle_openmp.py)."""
    lib = os.path.join(ROOT, "oracle", "liboracle_omp.so")
    if not os.path.exists(lib):
        return None
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    env = dict(os.environ, ORACLE_LIB=lib, OMP_NUM_THREADS=str(threads))
    nz = args.cpu_cols
    out = subprocess.run([sys.executable, "-c", PAR_SCRIPT, os.path.join(ROOT, "oracle"), str(Ny), str(nz),
                          str(N_min), str(N_max), str(args.seed), str(args.dt), str(args.cpu_calls)],
                         env=env, capture_output=True, text=True, check=True, timeout=600)
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    return {"value": Ny * nz / rec["s_per_call"], "unit": "cells/s", "cores": threads, "kind": "port",
            "sample": f"{Ny}x{nz} (as cpu_baseline), {args.cpu_calls} filter(dt) calls",
            "s_per_call": rec["s_per_call"],
            "note": "oracle restatement with OpenMP over the rows of the sweeps and elementwise steps "
                    "(RNG serial); not the reference, which is single-threaded"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("for --gpus > 1 launch with torch.distributed.run --nproc-per-node N")
        args.gpus = world

    # torch first: libdfamd.so then binds to the same HIP runtime torch loaded.
    import torch
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    sys.path.insert(0, PKG)
    import dfamd

    Ny, Nz_per, N_min, N_max, desc = CONFIGS[args.config]
    Nz = Nz_per * world
    comm_id = None
    if world > 1:
        obj = [dfamd.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]

    t_setup = time.perf_counter()
    f = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=N_min, N_max=N_max, seed=args.seed,
                            device=local_rank, rank=rank, world=world, comm_id=comm_id,
                            coeff_mode=args.coeff_mode, rows_per_wave=args.rows_per_wave)
    t_setup = time.perf_counter() - t_setup

    def barrier():
        if dist is not None:
            dist.barrier()

    def timed(h):
        """W untimed calls, then exactly K calls between barrier + synchronize; hipEvent phase profile."""
        for _ in range(args.warmup):
            h.filter(args.dt)
        h.sync()
        h.set_profiling(True)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            h.filter(args.dt)
        h.sync()
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        prof = h.profile()
        h.set_profiling(False)
        return el, prof

    elapsed, prof = timed(f)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    cells_total = Ny * Nz
    ms_per_step = elapsed * 1e3 / args.steps
    value = cells_total * args.steps / elapsed

    # roofline of the dominant kernel, from hipEvents on the library's stream
    phase = {"ypass": prof["ypass_ms"], "zpass": prof["zpass_ms"]}
    dom = max(phase, key=phase.get)
    dom_ms = phase[dom] / max(1, prof["calls"])
    alg = f.algorithmic_bytes(0 if dom == "ypass" else 1)
    call_alg = f.algorithmic_bytes(-1)
    achieved = alg / (dom_ms * 1e-3) / 1e9
    traffic = None
    traffic_src = None
    if os.path.exists(args.pmc_file):
        try:
            pm = json.load(open(args.pmc_file))
            key = f"{args.config}/{args.coeff_mode}/{dom}"
            if key in pm.get("per_launch_bytes", {}):
                traffic = pm["per_launch_bytes"][key]
                traffic_src = os.path.relpath(args.pmc_file, ROOT)
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "kernel": f"{dom}_kernel", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(dom_ms, 4)}
    if traffic_src:
        roofline["traffic_source"] = traffic_src
    # measured stream ceilings of this GPU model (tools/hbm_probe: 8 GiB grid-stride kernels)
    probe = os.path.join(ROOT, "profiles", "r1", "hbm_probe.json")
    if os.path.exists(probe):
        hp = json.load(open(probe))
        ceil = hp.get("read_nt_g8192_GBps")
        if ceil:
            roofline["measured_ceiling"] = {"nt_read_GBps": ceil, "copy_GBps": hp.get("copy_GBps"),
                                            "frac": round(achieved / ceil, 4),
                                            "source": os.path.relpath(probe, ROOT)}

    def load_pmc():
        try:
            return json.load(open(args.pmc_file)).get("per_launch_bytes", {})
        except Exception:
            return {}

    alt = None
    if world == 1 and args.alt_modes == "auto":
        other = "table" if args.coeff_mode == "packed" else "packed"
        f.close()
        g = dfamd.DigitalFilter(plane="synthetic", Ny=Ny, Nz=Nz, N_min=N_min, N_max=N_max, seed=args.seed,
                                device=local_rank, coeff_mode=other, rows_per_wave=args.rows_per_wave)
        taps = sum(g.comp_info(c)["by_size"] + g.comp_info(c)["bz_size"] for c in range(3))
        el2, p2 = timed(g)
        g.close()
        ms2 = el2 * 1e3 / args.steps
        pm = load_pmc()
        meas = [pm.get(f"{args.config}/{other}/{k}") for k in ("ypass", "zpass")]
        alt = {other: {"value": round(cells_total * args.steps / el2, 1), "ms_per_step": round(ms2, 4),
                       "phase_ms_per_call": {k: round(p2[k] / max(1, p2["calls"]), 4)
                                             for k in ("rng_ms", "ypass_ms", "halo_ms", "zpass_ms", "total_ms")}}}
        if other == "table":
            alt[other]["note"] = ("same results bit for bit (tests/test_gpu_parity.py); coefficients read from a "
                                  "per-N table instead of the 20.7 GB offset-packed stream, so SURVEY 8d's "
                                  "algorithmic bytes do not apply: the roofline uses rocprofv3-measured bytes")
            # Table mode is FP64-VALU bound: 2 flop (mul, add) per tap and cell (5.17 GFLOP at c3).
            # Peak: MI355X FP64 vector 78.6 TFLOP/s (datasheet; half the guide's 157.3 FP32); the sums
            # must not contract to FMA (bit-exactness), which caps mul+add at half of that.
            sw_ms = (p2["ypass_ms"] + p2["zpass_ms"]) / max(1, p2["calls"])
            flops = 2.0 * taps
            alt[other]["roofline_valu"] = {"bound": "valu-fp64", "achieved": round(flops / (sw_ms * 1e-3) / 1e12, 2),
                                           "peak": 78.6, "unit": "TFLOP/s",
                                           "frac": round(flops / (sw_ms * 1e-3) / 1e12 / 78.6, 4),
                                           "flops_per_call": flops, "sweeps_ms": round(sw_ms, 4),
                                           "note": "mul+add without FMA contraction caps at 39.3 TFLOP/s"}
            vp = os.path.join(ROOT, "profiles", "r1", "probe", "valu_probe_fp64.jsonl")
            if os.path.exists(vp):  # measured FP64 mul+add issue ceiling of this GPU model (tools/valu_probe)
                best = max(json.loads(l)["wave_instr_per_s"] for l in open(vp) if l.startswith("{"))
                ceil_tf = best * 64 / 1e12  # one flop per lane per v_mul_f64 / v_add_f64
                rv = alt[other]["roofline_valu"]
                rv["measured_ceiling"] = {"TFLOPs": round(ceil_tf, 1), "frac": round(rv["achieved"] / ceil_tf, 4),
                                          "source": os.path.relpath(vp, ROOT)}
            if all(m is not None for m in meas):
                sweeps_ms = (p2["ypass_ms"] + p2["zpass_ms"]) / max(1, p2["calls"])
                ach = sum(meas) / (sweeps_ms * 1e-3) / 1e9
                alt[other]["roofline_measured"] = {"bound": "hbm", "kernels": "ypass+zpass",
                                                   "measured_bytes_per_call": sum(meas),
                                                   "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS,
                                                   "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4),
                                                   "traffic_source": os.path.relpath(args.pmc_file, ROOT)}

    others = None
    if world == 1 and args.other_configs:
        # BASELINE configs[1] (c2, 512 x 512, N 4-32) and any others, same mode, same timing rule
        others = {}
        for name in filter(None, args.other_configs.split(",")):
            if name == args.config or name not in CONFIGS:
                continue
            oNy, oNz, olo, ohi, odesc = CONFIGS[name]
            h = dfamd.DigitalFilter(plane="synthetic", Ny=oNy, Nz=oNz, N_min=olo, N_max=ohi, seed=args.seed,
                                    device=local_rank, coeff_mode=args.coeff_mode, rows_per_wave=args.rows_per_wave)
            el3, p3 = timed(h)
            ph = {"ypass": p3["ypass_ms"], "zpass": p3["zpass_ms"]}
            d = max(ph, key=ph.get)
            d_ms = ph[d] / max(1, p3["calls"])
            d_ach = h.algorithmic_bytes(0 if d == "ypass" else 1) / (d_ms * 1e-3) / 1e9
            others[name] = {"workload": odesc, "value": round(oNy * oNz * args.steps / el3, 1),
                            "ms_per_step": round(el3 * 1e3 / args.steps, 4),
                            "phase_ms_per_call": {k: round(p3[k] / max(1, p3["calls"]), 4)
                                                  for k in ("rng_ms", "ypass_ms", "zpass_ms", "total_ms")},
                            "roofline": ({"kernel": f"{d}_kernel", "achieved": round(d_ach, 1), "unit": "GB/s",
                                          "frac": round(d_ach / HBM_PEAK_GBPS, 4)}
                                         if args.coeff_mode == "packed" else None)}
            h.close()

    out = None
    if rank == 0:
        cpu = cpu_par = None
        if args.cpu_baseline == "auto" and world == 1:
            try:
                cpu = cpu_baseline(args, Ny, N_min, N_max)
            except Exception as e:  # reported, never fatal for the GPU number
                cpu = {"error": str(e)}
            try:
                cpu_par = cpu_baseline_parallel(args, Ny, N_min, N_max)
            except Exception as e:
                cpu_par = {"error": str(e)}
        per_call = {k: round(prof[k] / max(1, prof["calls"]), 4) for k in ("rng_ms", "ypass_ms", "halo_ms",
                                                                            "zpass_ms", "total_ms")}
        out = {
            "metric": "inflow cells/sec (filter(dt) call) + achieved HBM GB/s, 1/2/4/8 GPU",
            "value": round(value, 1),
            "unit": "cells/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY 8d plane; rows from files/RST.dat + line.dat; pcg32 seed %d)" % args.seed,
            "config": {"workload": desc, "Ny": Ny, "Nz": Nz, "N_min": N_min, "N_max": N_max,
                       "dt": args.dt, "coeff_mode": args.coeff_mode, "rows_per_wave": args.rows_per_wave,
                       "parallelism": f"z-strips x{world}" if world > 1 else "single GPU"},
            "achieved_call_GBps": round(call_alg / (ms_per_step * 1e-3) / 1e9 * world, 1),
            "call_hbm_frac": round(call_alg * world / (ms_per_step * 1e-3) / 1e9 / (HBM_PEAK_GBPS * world), 4),
            "phase_ms_per_call": per_call,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_baseline_parallel": cpu_par,
            "alt_modes": alt,
            "other_configs": others,
            "setup_s": round(t_setup, 3),
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if world > 1 or args.alt_modes == "off":
        f.close()


if __name__ == "__main__":
    main()
