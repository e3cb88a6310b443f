#!/usr/bin/env python3
"""Benchmark of DIGITAL_FILTER::filter(dt) on MI355X (BASELINE.json metric).

One step = one filter(dt) call (reference df.cpp:449-468) over the whole plane:
device RNG in the reference's stream order, y- and z-convolutions streaming the
offset-packed coefficients, correlation, RST scaling, SRA T'/rho'.

Workloads (BASELINE.json configs; SURVEY 8d half-width rule, dt = 1e-8):
  c3  2048 x 2048, N 4-64      configs[2], the HBM roofline point: the N = 1 default
  c4  2048 x 8192, N 4-64      configs[3]: split into N z-strips, the N > 1 default
  c5  4096 x 4096, N 4-64      configs[4]: split into N z-strips (reported beside c4 at N > 1)
  c2  512 x 512, N 4-32        configs[1];  c1 128 x 128, N = 8 (configs[0], the CPU case)
  native                       the reference's own 510 x 400 grid (df.cpp:71-118)
--scaling strong (default) keeps the plane and splits it over the ranks; --scaling weak gives
every rank the config's whole plane as its strip (plane Nz x N). Multi-GPU: one process per
GPU, one RCCL halo exchange per call; after the timed region every rank re-runs the whole
plane unsplit in table mode on its own GPU and compares its strip bit for bit (parity_ok).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--coeff-mode packed|table]
    torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` with N > 1 outside a torchrun launch starts one itself: before torch is
imported or any GPU touched, it runs `python -m torch.distributed.run --nproc-per-node N bench.py
...` as a CHILD process (never exec), relays rank 0's JSON line to stdout and exits with the
child's return code. At N > 1 rank 0 also times the whole plane unsplit on its own GPU after the
timed region (`same_plane_1gpu`: the 1-GPU time of the SAME plane, and the speedup over it), and
the c5 line runs BASELINE configs[4]'s 10 000 filter(dt) steps for real (`long_run`).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "digital-filtering_amd")
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FIELDS = ("u", "v", "w", "T", "rho")
RNG_COLLECTIVE = {  # df_comm_stats.rng_collective (include/df_c.h)
    0: "none: every rank counts the whole stream (replicated), halo is the only collective",
    1: "allgather: share records (per-64-attempt accept counts) on a second communicator",
    2: "in the halo group: share records of a later generation ride in the call's ncclGroup (one grouped op per call)",
}

# name: plane, Ny, Nz (whole plane), N_min, N_max, description
CONFIGS = {
    "c1": ("synthetic", 128, 128, 8, 8, "c1: 128x128 plane, constant half-width N=8"),
    "c2": ("synthetic", 512, 512, 4, 32, "c2: 512x512 plane, half-width 4-32"),
    "c3": ("synthetic", 2048, 2048, 4, 64, "c3: 2048x2048 plane, half-width 4-64 (HBM roofline point)"),
    "c4": ("synthetic", 2048, 8192, 4, 64, "c4: 2048x8192 plane, half-width 4-64, z-strips over the GPUs"),
    "c5": ("synthetic", 4096, 4096, 4, 64, "c5: 4096x4096 plane, half-width 4-64, z-strips over the GPUs"),
    "native": ("native", 0, 0, 0, 0, "native: the reference's own 510x400 grid (read_grid, df.cpp:71-118)"),
}


def plan_workload(name, world, scaling="strong"):
    """The plane one run times and each rank's z-strip [z0, z1) (df_capi.cpp plan_strips:
    z0 = r*Nz/world). strong: the config's plane split over the ranks; weak: a plane Nz*world
    wide, so every rank holds the config's Nz columns."""
    plane, Ny, Nz, lo, hi, desc = CONFIGS[name]
    if plane == "native":
        if world > 1:
            raise ValueError("the native grid is a single-GPU plane")
        return {"name": name, "plane": plane, "Ny": 510, "Nz": 400, "N_min": 0, "N_max": 0, "desc": desc,
                "scaling": "strong", "strips": [(0, 400)]}
    if scaling not in ("strong", "weak"):
        raise ValueError(scaling)
    Nzg = Nz * world if scaling == "weak" else Nz
    strips = [(r * Nzg // world, (r + 1) * Nzg // world) for r in range(world)]
    if world > 1 and min(z1 - z0 for z0, z1 in strips) < hi:
        raise ValueError(f"{name} over {world} GPUs: strips narrower than the z half-width {hi}")
    if scaling == "weak" and world > 1:
        desc = f"{desc.split(':')[0]} per GPU (weak): {Ny}x{Nzg} plane, {Ny}x{Nz} per GPU, half-width {lo}-{hi}"
    return {"name": name, "plane": plane, "Ny": Ny, "Nz": Nzg, "N_min": lo, "N_max": hi, "desc": desc,
            "scaling": scaling if world > 1 else "strong", "strips": strips}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="auto", choices=["auto"] + sorted(CONFIGS),
                   help="auto: c3 on one GPU, c4 split over N > 1 GPUs")
    p.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    p.add_argument("--coeff-mode", default="packed", choices=["packed", "table"])
    p.add_argument("--rows-per-wave", type=int, default=0)  # 0 = library default per mode
    p.add_argument("--dt", type=float, default=1e-8)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--parity", default="on", choices=["on", "off"],
                   help="after the timed region compare every rank's strip with the unsplit plane (table mode)")
    p.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    p.add_argument("--cpu-full-cols", type=int, default=0,
                   help="columns of the reference CPU run (0: the GPU plane's own, i.e. the whole plane)")
    p.add_argument("--cpu-calls", type=int, default=3)  # c3: ~15 s of reference CPU work (5 s per call)
    p.add_argument("--cpu-cols", type=int, default=512,
                   help="columns of the secondary CPU sample (same rows and rule; 0: none)")
    p.add_argument("--cpu-sample-calls", type=int, default=6)
    p.add_argument("--pmc-file", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--other-configs", default="auto",
                   help="comma list of further configs timed after the main one, same mode and rule; "
                        "auto: 'native,c2' on one GPU, 'c5' on N > 1; '' for none")
    p.add_argument("--alt-modes", default="auto", choices=["auto", "off"],
                   help="also time the other coefficient mode (at N > 1 split the same way) and report it under alt_modes")
    p.add_argument("--same-plane", default="auto", choices=["auto", "off"],
                   help="N > 1: rank 0 also times the whole plane unsplit on its own GPU (same_plane_1gpu)")
    p.add_argument("--long-run", default="auto",
                   help="filter(dt) calls of the long run (device get_rms accumulation every call, steady-state "
                        "and total time, the SURVEY 4 variance invariant at the end); auto: 10000 on c5 at N > 1 "
                        "(BASELINE configs[4]), else none; an integer K runs K calls on the main workload")
    p.add_argument("--profile-every", type=int, default=4,
                   help="phase events (hipEventRecord) on every n-th timed call only: on calls of 0.1-0.2 ms six "
                        "events per call cost 1-10%% of the wall time (tools/event_cost.py)")
    p.add_argument("--dry-run", action="store_true",
                   help="launch plumbing only: every rank reports its env, rank 0 prints one JSON line; no GPU")
    p.add_argument("--dropin", default="auto", choices=["auto", "off"],
                   help="N=1: time the C++ drop-in (examples/cpp-test) DIGITAL_FILTER::filter() wall per call")
    a = p.parse_args(argv)
    return a


def progress(msg):
    """Progress on stderr (stdout carries only the JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_command(argv, n, port):
    """The torchrun command a bare `bench.py --gpus N` (N > 1) starts as its child: one rank per GPU
    of this node, rendezvous on 127.0.0.1, the same bench arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


PROGRESS_ENV = "DFAMD_PROGRESS_DIR"
LAUNCH_TIMEOUT_S = 1500  # the whole N-rank job; a bare 8-GPU run takes a few minutes (profiles/r4/j: 515 s with emulated hosts)


def rank_phase(name, rank=None):
    """Record this rank's current phase (create, warm-up, timed, parity, same-plane, long-run, ...) in
    $DFAMD_PROGRESS_DIR/rank<r>.log, one timestamped line per phase, so a launch that hangs or dies says
    where each rank stopped (the parent prints the files on failure)."""
    d = os.environ.get(PROGRESS_ENV)
    if not d:
        return
    r = int(os.environ.get("RANK", "0")) if rank is None else rank
    try:
        with open(os.path.join(d, f"rank{r}.log"), "a") as fh:
            fh.write(f"{time.strftime('%H:%M:%S')} {time.monotonic():.3f} {name}\n")
    except OSError:
        pass


def report_progress(d):
    """Each rank's last recorded phases (stderr): where a failed or timed-out launch stopped."""
    try:
        names = sorted(x for x in os.listdir(d) if x.startswith("rank") and x.endswith(".log"))
    except OSError:
        names = []
    if not names:
        progress(f"no rank recorded a phase in {d}")
    for nm in names:
        lines = open(os.path.join(d, nm)).read().splitlines()
        progress(f"{nm[:-4]}: last phase '{lines[-1].split(' ', 2)[-1] if lines else '-'}' "
                 f"({len(lines)} recorded: {', '.join(l.split(' ', 2)[-1] for l in lines[-6:])})")


def self_launch(argv, n, cmd=None, timeout_s=None):
    """Run the N-rank bench as a child process (never os.exec*: this process has not touched the GPU
    and must not replace itself), relay its JSON line (the one rank 0 prints) to stdout and everything
    else to stderr, and return the child's return code (1 if it succeeded without a JSON line).

    The child gets a wall-clock budget (timeout_s, default $DFAMD_BENCH_TIMEOUT or LAUNCH_TIMEOUT_S): on
    expiry its whole process group (torchrun and every rank) is terminated, then killed, and the launch
    returns 124. Every rank records its phases under $DFAMD_PROGRESS_DIR (a fresh directory unless set);
    on any failure the parent prints each rank's last phase."""
    import shutil
    import signal
    import tempfile
    import threading

    cmd = cmd or launch_command(argv, n, free_port())
    if timeout_s is None:
        timeout_s = float(os.environ.get("DFAMD_BENCH_TIMEOUT", LAUNCH_TIMEOUT_S))
    own_dir = PROGRESS_ENV not in os.environ
    pdir = os.environ.get(PROGRESS_ENV) or tempfile.mkdtemp(prefix="dfamd_bench_progress_")
    env = dict(os.environ, **{PROGRESS_ENV: pdir})
    progress(f"launching (budget {timeout_s:.0f} s, rank phases in {pdir}): " + " ".join(cmd))
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1, env=env, start_new_session=True)
    expired = threading.Event()

    def expire():
        expired.set()
        progress(f"wall-clock budget of {timeout_s:.0f} s exceeded: terminating the ranks")
        for sig, wait in ((signal.SIGTERM, 10.0), (signal.SIGKILL, 0.0)):
            try:
                os.killpg(proc.pid, sig)
            except ProcessLookupError:
                return
            try:
                proc.wait(wait)
                return
            except subprocess.TimeoutExpired:
                pass

    timer = threading.Timer(timeout_s, expire)
    timer.daemon = True
    timer.start()
    line_out = None
    interrupted = None

    class Interrupted(Exception):
        pass

    # the ranks run in their own session, so a SIGTERM / SIGINT / SIGHUP meant for this launcher
    # (an outer `timeout`, Ctrl-C, a closed terminal) would not reach them. Turn it into an exception here so
    # the finally block below ends their process group before this process exits.
    def on_signal(signum, frame):
        raise Interrupted(signum)

    handled = (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)
    previous = {sig: signal.signal(sig, on_signal) for sig in handled}
    rc = 1
    try:
        for line in proc.stdout:
            st = line.strip()
            if st.startswith("{") and '"metric"' in st:
                line_out = st
                print(st, flush=True)
            else:
                sys.stderr.write(line)
                sys.stderr.flush()
        rc = proc.wait()
    except Interrupted as e:
        interrupted = e.args[0]
        progress(f"signal {interrupted} received: terminating the ranks")
    finally:
        timer.cancel()
        for sig in handled:  # no second handler run while the group is being ended
            signal.signal(sig, signal.SIG_IGN)
        if proc.poll() is None:
            for sig, wait in ((signal.SIGTERM, 10.0), (signal.SIGKILL, 5.0)):
                try:
                    os.killpg(proc.pid, sig)
                    proc.wait(wait)
                    break
                except ProcessLookupError:
                    break
                except subprocess.TimeoutExpired:
                    pass
        for sig, h in previous.items():
            signal.signal(sig, h)
    if interrupted is not None:
        rc = 128 + int(interrupted)
    elif expired.is_set():
        rc = 124
    elif rc == 0 and line_out is None:
        progress("the launched ranks exited 0 without a JSON line")
        rc = 1
    if rc != 0:
        report_progress(pdir)
    if own_dir and rc == 0:
        shutil.rmtree(pdir, ignore_errors=True)
    return rc


def host_cpu():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"host_cpu": model, "host_cores": os.cpu_count(), "host_cores_usable": usable,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def ref_time(args, Ny, Nz, N_min, N_max, calls, timeout=1200):
    """The reference itself (oracle/_ref/ref_harness `time`: df.cpp built from the reference sources with
    g++ -O2, one thread) on an Ny x Nz plane of the SURVEY 8d rule: construction, then `calls` filter(dt)
    calls minus the CSV write - the region of the reference's own timer (df.cpp:452-462). None when the
    harness was not built (the box only has what this container built)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    run_root = os.path.join(ROOT, "oracle", "_ref", "run_root")
    if not (os.path.exists(exe) and os.path.isdir(run_root)):
        return None
    out = subprocess.run([exe, "time", run_root, str(args.seed), str(Ny), str(Nz), str(N_min), str(N_max),
                          str(args.dt), str(calls)], capture_output=True, text=True, check=True, timeout=timeout)
    return json.loads(out.stdout.strip().splitlines()[-1])


def cpu_baseline(args, Ny, Nz, N_min, N_max):
    """Reference CPU path on this host, on the WHOLE plane the GPU line times: df.cpp
    built from the reference sources (oracle/_ref/ref_harness, g++ -O2, 1 thread), `--cpu-calls` calls
    (c3: ~5 s each after a ~1 min construction holding 21 GB of host coefficients); else the oracle
    restatement. A narrower sample (`--cpu-cols` columns, same rows and rule) is timed beside it, and the
    sample/whole ratio of cells/s is the measured check of the per-cell extrapolation to c4/c5."""
    nz = Nz if args.cpu_full_cols <= 0 else args.cpu_full_cols
    sample = (f"the whole {Ny}x{nz} plane (the GPU line's rows, columns and N {N_min}-{N_max} rule), "
              f"{args.cpu_calls} filter(dt) calls after construction")
    rec = ref_time(args, Ny, nz, N_min, N_max, args.cpu_calls)
    if rec is not None:
        res = {"value": Ny * nz / rec["mean_s"], "unit": "cells/s", "cores": 1, "kind": "reference",
               "sample": sample, "s_per_call": rec["mean_s"], "best_s_per_call": rec["best_s"],
               "construction_s": rec["setup_s"],
               "stage_s": {k: rec[k] for k in ("noise_s", "sweeps_s", "correlate_s", "rst_s", "sra_s")}}
        if args.cpu_cols > 0 and args.cpu_cols < nz:
            sm = ref_time(args, Ny, args.cpu_cols, N_min, N_max, args.cpu_sample_calls)
            sm_rate = Ny * args.cpu_cols / sm["mean_s"]
            res["column_sample"] = {
                "sample": f"{Ny}x{args.cpu_cols}, {args.cpu_sample_calls} calls", "value": round(sm_rate, 1),
                "s_per_call": sm["mean_s"], "sample_over_whole": round(sm_rate / res["value"], 4),
                "note": "cells/s of a narrower plane of the same rows and rule over the whole plane's: "
                        "1.0 means the per-cell cost is column-independent (the c4/c5 extrapolation's premise)"}
    else:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=Ny, Nz=nz, N_min=N_min, N_max=N_max, seed=args.seed)
        t0 = time.perf_counter()
        for _ in range(args.cpu_calls):
            o.filter(args.dt)
        dt = (time.perf_counter() - t0) / args.cpu_calls
        res = {"value": Ny * nz / dt, "unit": "cells/s", "cores": 1, "kind": "port", "sample": sample,
               "s_per_call": dt}
    res.update(host_cpu())
    # BASELINE.md CPU plan step 5: the multi-GPU configs per cell from this plane (derived, not run)
    res["extrapolated"] = {
        name: {"cells": CONFIGS[name][1] * CONFIGS[name][2],
               "s_per_call": round(CONFIGS[name][1] * CONFIGS[name][2] / res["value"], 3),
               "derived": "cells / the whole plane's cells/s (same N rule; column_sample checks the per-cell premise)"}
        for name in ("c4", "c5")}
    return res


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
                          str(N_min), str(N_max), str(args.seed), str(args.dt), str(args.cpu_sample_calls)],
                         env=env, capture_output=True, text=True, check=True, timeout=600)
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    return {"value": Ny * nz / rec["s_per_call"], "unit": "cells/s", "cores": threads, "kind": "port",
            "sample": f"{Ny}x{nz} (cpu_baseline's column sample), {args.cpu_sample_calls} filter(dt) calls",
            "s_per_call": rec["s_per_call"],
            "note": "oracle restatement with OpenMP over the rows of the sweeps and elementwise steps "
                    "(RNG serial); not the reference, which is single-threaded"}


def dropin_timing(args):
    """The C++ drop-in's per-call cost: examples/cpp-test `time` runs, on one
    object, the C-ABI call with the per-step wait a synchronous caller makes (df_filter + df_wait: this call's
    fields; `capi_sync_all_ms`: + df_sync, which also waits for later calls' noise and y-passes), the same with
    the y-pass-ahead setting flipped, and DIGITAL_FILTER::filter() with host_mirror 0 (no host copies; also
    stream-ordered, no host wait), 1 (default: u/v/w.fluc, T', rho' - one sync, page-locked vectors) and 2
    (also filt_old and filt), on the reference's grid and on c3, in both coefficient modes. The mirror refresh
    is a PCIe D2H transfer of 5 (or 8) fields; `mirror1_GBps` is its rate."""
    exe = os.path.join(ROOT, "examples", "cpp-test")
    if not os.path.exists(exe):
        return {"error": "examples/cpp-test not built (make -C examples)"}
    out = {}
    for plane, dims in (("native", ("0", "0", "0", "0")), ("c3", ("2048", "2048", "4", "64"))):
        for mode in ("table", "packed"):
            progress(f"drop-in timing {plane} {mode}")
            try:
                r = subprocess.run([exe, "time", "native" if plane == "native" else "synth", *dims, mode, "60"],
                                   capture_output=True, text=True, timeout=300, check=True)
                rec = json.loads(r.stdout.strip().splitlines()[-1])
                d = rec["dropin_ms"]
                extra = d["mirror1"] - d["mirror0"]
                rec["mirror1_GBps"] = round(rec["mirror_bytes"]["mirror1"] / (extra * 1e-3) / 1e9, 1) if extra > 0 else None
                rec["dropin_over_capi"] = round(d["mirror1"] / rec["capi_ms"], 3)
                out[f"{plane}/{mode}"] = rec
            except Exception as e:  # reported, never fatal for the GPU number
                out[f"{plane}/{mode}"] = {"error": str(e)[-400:]}
    return out


class Ctx:
    """Process-group plumbing: rank, world, device and the gather/reduce helpers."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.device = self.local_rank
        # DFAMD_EMULATE_HOSTS=1: a rehearsal of the N-GPU path on one GPU. Every rank uses device 0 and
        # names its own host to RCCL (NCCL_HOSTID), whose duplicate-GPU check is per host; the ranks then
        # talk through RCCL's socket transport on the loopback interface instead of xGMI. Same product
        # calls, different transport: for checking the multi-GPU path, never for a scaling number.
        self.emulated = os.environ.get("DFAMD_EMULATE_HOSTS", "0") == "1" and self.world > 1
        if self.emulated:
            self.device = 0
            os.environ.update(NCCL_HOSTID=f"dfamd-emulated-host-{self.rank}", NCCL_SOCKET_IFNAME="lo",
                              NCCL_IB_DISABLE="1", NCCL_NET="Socket")
        self.dist = None

    def init(self, torch, backend="nccl"):
        """backend "nccl" (RCCL, the bench) or "gloo" (CPU tests of this plumbing)."""
        self.torch = torch
        if backend == "nccl":
            torch.cuda.set_device(self.device)
        if self.world > 1:
            import torch.distributed as dist
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.device))
            else:
                dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def comm_id(self, dfamd):
        if self.dist is None:
            return None
        obj = [dfamd.comm_unique_id() if self.rank == 0 else None]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]


def make_filter(dfamd, ctx, wl, args, coeff_mode, split=True, comm_id=None):
    kw = dict(seed=args.seed, device=ctx.device, coeff_mode=coeff_mode, rows_per_wave=args.rows_per_wave)
    if wl["plane"] == "native":
        return dfamd.DigitalFilter(plane="native", **kw)
    kw.update(plane="synthetic", Ny=wl["Ny"], Nz=wl["Nz"], N_min=wl["N_min"], N_max=wl["N_max"])
    if split and ctx.world > 1:
        kw.update(rank=ctx.rank, world=ctx.world, comm_id=comm_id)
    return dfamd.DigitalFilter(**kw)


def timed(ctx, h, args, min_warm_s=0.0, profile=True, collective=True, label=""):
    """W untimed calls, then exactly K calls between barrier + synchronize; hipEvent phase profile.
    min_warm_s > 0 (secondary lines only: alt mode, other configs) keeps warming up until that much
    time has passed: a 0.4 ms table-mode call otherwise starts timing while the clocks still ramp
    (c3 table: 0.395 ms/call after 5 calls, 0.370 after 140; profiles/r2/table_warmup.txt)."""
    torch = ctx.torch
    calls = 0
    rank_phase(f"{label}: warm-up ({args.warmup} calls)")
    for _ in range(args.warmup):
        h.filter(args.dt)
        calls += 1
    h.sync()
    t_w = time.perf_counter()
    # one process only: every call of a split plane is an RCCL exchange, so ranks must run equal counts
    while min_warm_s > 0 and (ctx.world == 1 or not collective) and time.perf_counter() - t_w < min_warm_s:
        for _ in range(10):
            h.filter(args.dt)
            calls += 1
        h.sync()
    h.set_profiling(profile, every=args.profile_every if args.steps >= 2 * args.profile_every else 1)
    rank_phase(f"{label}: timed ({args.steps} calls)")
    if collective:
        ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        h.filter(args.dt)
    h.sync()
    torch.cuda.synchronize()
    if collective:
        ctx.barrier()
    el = time.perf_counter() - t0
    prof = h.profile() if profile else None
    h.set_profiling(False)
    return el, prof, calls + args.steps


def per_call(prof):
    return {k: round(prof[k] / max(1, prof["calls"]), 4) for k in ("rng_ms", "ypass_ms", "halo_ms", "zpass_ms",
                                                                 "total_ms")}


def compare(h, ref, z0, z1):
    """Bit-for-bit comparison of this strip with the same columns of the unsplit plane."""
    bad = {}
    worst = 0.0
    for k in FIELDS:
        a = h.field(k)
        b = np.ascontiguousarray(ref.field(k)[:, z0:z1])
        n = int(np.count_nonzero(a.view(np.uint64) != b.view(np.uint64)))
        if n:
            bad[k] = n
            worst = max(worst, float(np.nanmax(np.abs(a - b))))
    rng_ok = h.rng_state() == ref.rng_state()
    return {"ok": (not bad) and rng_ok, "mismatched_cells": bad, "max_abs_diff": worst, "rng_state_equal": rng_ok}


def parity_check(dfamd, ctx, wl, args, h, calls, ref=None):
    """This rank's strip after construction + `calls` filter(dt) calls against the whole plane run unsplit in table mode
    on this rank's own GPU (packed and table mode, any strip count: bit-identical by construction)."""
    own = ref is None
    rank_phase(f"{wl['name']}: parity (whole plane unsplit, table mode)")
    if own:
        ref = make_filter(dfamd, ctx, wl, args, "table", split=False)
        for _ in range(calls):
            ref.filter(args.dt)
    z0, z1 = h.z0, h.z1
    res = compare(h, ref, z0, z1)
    if own:
        ref.close()
    res["rank"] = ctx.rank
    res["columns"] = [z0, z1]
    return res


def roofline_of(h, prof, args, config_name):
    phase = {"ypass": prof["ypass_ms"], "zpass": prof["zpass_ms"]}
    dom = max(phase, key=phase.get)
    dom_ms = phase[dom] / max(1, prof["calls"])
    alg = h.algorithmic_bytes(0 if dom == "ypass" else 1)
    achieved = alg / (dom_ms * 1e-3) / 1e9
    r = {"bound": "hbm", "kernel": f"{dom}_kernel", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
         "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(dom_ms, 4)}
    if os.path.exists(args.pmc_file):
        try:
            pm = json.load(open(args.pmc_file)).get("per_launch_bytes", {})
            key = f"{config_name}/{args.coeff_mode}/{dom}"
            if key in pm:
                r["traffic"] = pm[key]
                r["traffic_source"] = os.path.relpath(args.pmc_file, ROOT)
        except Exception:
            pass
    probe = os.path.join(ROOT, "profiles", "r1", "hbm_probe.json")
    if os.path.exists(probe):  # measured stream ceilings of this GPU model (tools/hbm_probe)
        hp = json.load(open(probe))
        ceil = hp.get("read_nt_g8192_GBps")
        if ceil:
            r["measured_ceiling"] = {"nt_read_GBps": ceil, "copy_GBps": hp.get("copy_GBps"),
                                     "frac": round(achieved / ceil, 4), "source": os.path.relpath(probe, ROOT)}
    return r


def run_config(dfamd, ctx, wl, args, comm_id, min_warm_s=0.0):
    """Create and time one workload on every rank; returns the handle and this rank's record."""
    rank_phase(f"{wl['name']}: create (df_create, step 0)")
    t_setup = time.perf_counter()
    f = make_filter(dfamd, ctx, wl, args, args.coeff_mode, comm_id=comm_id)
    t_setup = time.perf_counter() - t_setup
    elapsed, prof, ncalls = timed(ctx, f, args, min_warm_s, label=wl["name"])
    f.calls_done = ncalls  # filter(dt) calls after step 0, for the parity reference
    rank_rec = {"rank": ctx.rank, "elapsed_s": elapsed, "phase_ms_per_call": per_call(prof),
                "roofline": roofline_of(f, prof, args, wl["name"]), "columns": [f.z0, f.z1],
                "comm": f.comm_info() if ctx.world > 1 else None, "setup_s": round(t_setup, 3),
                "call_bytes": f.algorithmic_bytes(-1)}
    return f, rank_rec


def same_plane_1gpu(dfamd, ctx, wl, args, split_ms):
    """N > 1, rank 0: the whole plane unsplit on its own GPU, same mode, K and W, after every rank has
    closed its strip: the 1-GPU time of the SAME plane the N ranks split, and the speedup over it.
    The other ranks wait at the barrier. (near-linear vs 1 GPU on one plane.)"""
    res = None
    rank_phase(f"{wl['name']}: same-plane baseline ({'timing' if ctx.rank == 0 else 'waiting at the barrier'})")
    if ctx.rank == 0:
        progress(f"{wl['name']}: whole plane on one GPU (same-plane baseline)")
        h = make_filter(dfamd, ctx, wl, args, args.coeff_mode, split=False)
        el, prof, _ = timed(ctx, h, args, collective=False)
        roof = roofline_of(h, prof, args, wl["name"])
        h.close()
        ms = el * 1e3 / args.steps
        res = {"ms_per_step": round(ms, 4), "value": round(wl["Ny"] * wl["Nz"] * args.steps / el, 1),
               "phase_ms_per_call": per_call(prof), "roofline_frac": roof["frac"],
               "speedup": round(ms / split_ms, 3),
               "note": "rank 0 alone, whole plane unsplit on its GPU after the timed region; speedup = this "
                       "ms_per_step / the N-rank ms_per_step (max over ranks)"}
    ctx.barrier()
    return res


def long_run(dfamd, ctx, wl, args, steps, comm_id):
    """BASELINE configs[4]'s run for real: `steps` filter(dt) calls, each followed by the device
    get_rms accumulation (df.cpp:584-611: filter, then rms_add), timed as a whole (barrier +
    synchronize on both sides, max over ranks) and in windows of steps/10 calls (steady state). At the
    end, SURVEY 4's invariant over the whole plane: per row, the mean of u'^2, v'^2, w'^2 over time
    and every rank's columns against R11, R22, R33 (rows with R11 > 1% of its max)."""
    torch = ctx.torch
    rank_phase(f"{wl['name']}: long run ({steps} calls)")
    h = make_filter(dfamd, ctx, wl, args, args.coeff_mode, comm_id=comm_id)
    h.filter(args.dt)
    h.sync()
    h.rms_reset()
    win = max(1, steps // 10)
    windows = []
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = last = time.perf_counter()
    for i in range(steps):
        h.filter(args.dt)
        h.rms_add()
        if (i + 1) % win == 0 or i + 1 == steps:
            h.sync()
            now = time.perf_counter()
            n = (i + 1) - (len(windows) * win)
            windows.append(round((now - last) * 1e3 / n, 4))
            last = now
            if ctx.rank == 0:
                progress(f"long run {wl['name']}: {i + 1}/{steps} calls, {windows[-1]} ms/call")
    h.sync()
    torch.cuda.synchronize()
    ctx.barrier()
    total = time.perf_counter() - t0
    sums = {k: (h.rms(k) ** 2).sum(axis=1) for k in ("u", "v", "w")}  # per row, this strip's columns
    rows = {k: h.row(k) for k in ("R11", "R22", "R33")}
    finite = bool(all(np.isfinite(h.field(k)).all() for k in FIELDS))
    state = h.rng_state()
    h.close()
    recs = ctx.gather({"total_s": total, "windows": windows, "sums": sums, "finite": finite,
                       "rng_state": [str(state[0]), int(state[1])]})
    if ctx.rank != 0:
        return None
    R = rows
    mask = R["R11"] > 0.01 * R["R11"].max()
    dev = {}
    for name, r in (("u", "R11"), ("v", "R22"), ("w", "R33")):
        ms2 = sum(x["sums"][name] for x in recs) / wl["Nz"]
        dev[name] = round(float(np.abs(ms2[mask] / R[r][mask] - 1).max()), 4)
    tot = max(x["total_s"] for x in recs)
    steady = [max(x["windows"][i] for x in recs) for i in range(len(recs[0]["windows"]))]
    return {"steps": steps, "total_s": round(tot, 3), "ms_per_call_incl_rms": round(tot * 1e3 / steps, 4),
            "steady_ms_per_call": round(float(np.median(steady[1:] if len(steady) > 1 else steady)), 4),
            "window_ms_per_call": steady, "window_calls": win,
            "max_rel_dev_rowvar_vs_R": dev, "rows_checked": int(mask.sum()),
            "fields_finite": all(x["finite"] for x in recs),
            "rng_state_equal_on_ranks": len({tuple(x["rng_state"]) for x in recs}) == 1,
            "note": "every call = filter(dt) + rms_add on the device (the reference's get_rms loop, "
                    "df.cpp:596-606); times max over ranks; windows of window_calls calls"}


def summarize(ctx, wl, args, recs):
    """Whole-job numbers from every rank's record (max-over-ranks time)."""
    el_max = max(r["elapsed_s"] for r in recs)
    el_min = min(r["elapsed_s"] for r in recs)
    cells = wl["Ny"] * wl["Nz"]
    ms = el_max * 1e3 / args.steps
    slowest = max(recs, key=lambda r: r["roofline"]["avg_launch_ms"])
    out = {"value": round(cells * args.steps / el_max, 1), "ms_per_step": round(ms, 4),
           "phase_ms_per_call": recs[0]["phase_ms_per_call"], "roofline": slowest["roofline"]}
    if ctx.world > 1:
        out["roofline"] = dict(slowest["roofline"], rank=slowest["rank"],
                               frac_by_rank=[r["roofline"]["frac"] for r in recs])
    if args.coeff_mode == "packed" and all(r.get("call_bytes") for r in recs):
        # the whole call's algorithmic bytes (y- and z-pass) over the wall per call: where the y-pass
        # runs ahead it shares the chip with the z-pass, and the kernel figure above counts only its own bytes
        cb = sum(r["call_bytes"] for r in recs)
        gbs = cb / (ms * 1e-3) / 1e9
        out["roofline"] = dict(out["roofline"], call={
            "bytes": cb, "ms": round(ms, 4), "achieved": round(gbs, 1),
            "frac": round(gbs / (HBM_PEAK_GBPS * ctx.world), 4),
            "note": "every sweep's algorithmic bytes of one call / ms_per_step (all ranks) / the peak of all ranks"})
    if ctx.world > 1:
        cm = recs[0]["comm"] or {}
        out["multi_gpu"] = {
            "rccl_ranks": cm.get("rccl_ranks"),
            "rng_collective": RNG_COLLECTIVE.get(cm.get("rng_collective", 0), "?"),
            "halo_ms_per_call": {"max": max(r["phase_ms_per_call"]["halo_ms"] for r in recs),
                                 "min": min(r["phase_ms_per_call"]["halo_ms"] for r in recs)},
            "halo_bytes_per_call": sum((r["comm"] or {}).get("halo_bytes_sent", 0) for r in recs),
            "rng_collective_bytes_per_call": sum((r["comm"] or {}).get("rng_bytes_received", 0) for r in recs),
            "rank_ms_per_step": {"min": round(el_min * 1e3 / args.steps, 4), "max": round(ms, 4)},
            "per_rank": [{"rank": r["rank"], "columns": r["columns"],
                          "ms_per_step": round(r["elapsed_s"] * 1e3 / args.steps, 4),
                          "phase_ms_per_call": r["phase_ms_per_call"]} for r in recs],
        }
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # a bare `bench.py --gpus N`: start the N ranks as a child torchrun (torch not imported yet)
        return self_launch(argv, args.gpus)
    ctx = Ctx()
    if args.dry_run:  # tests/test_bench_launch.py: the self-launch reaches N ranks with the right env
        rank_phase("dry-run", ctx.rank)
        if ctx.rank == 0:
            print(json.dumps({"metric": "dry-run", "n_gpus": ctx.world, "gpus_arg": args.gpus,
                              "master_addr": os.environ.get("MASTER_ADDR"), "argv": argv}), flush=True)
        return 0
    if ctx.world != args.gpus:
        args.gpus = ctx.world
    name = args.config if args.config != "auto" else ("c3" if ctx.world == 1 else "c4")
    wl = plan_workload(name, ctx.world, args.scaling)
    others_arg = args.other_configs
    if others_arg == "auto":
        others_arg = "native,c2,c1" if ctx.world == 1 else "c5"

    # torch first: libdfamd.so then binds to the same HIP runtime torch loaded.
    rank_phase("init: torch + process group", ctx.rank)
    import torch
    ctx.init(torch)
    sys.path.insert(0, PKG)
    import dfamd

    comm_id = ctx.comm_id(dfamd)
    if ctx.rank == 0:
        progress(f"{name}: {wl['Ny']}x{wl['Nz']} over {ctx.world} rank(s), {args.coeff_mode}")
    f, rec = run_config(dfamd, ctx, wl, args, comm_id)
    recs = ctx.gather(rec)
    head = summarize(ctx, wl, args, recs)
    # the headline handle's parity, then close it: the other mode's line below is timed without it resident beside
    # (an idle handle's streams still take hardware queues)
    parity = None
    if args.parity == "on":
        pr = parity_check(dfamd, ctx, wl, args, f, f.calls_done)
        prs = ctx.gather(pr)
        parity = {"ok": all(p["ok"] for p in prs), "reference": "whole plane, one GPU, table mode, same seed/calls",
                  "calls_compared": f.calls_done, "ranks": prs if ctx.world > 1 else prs[0]}
    comm = f.comm_info() if ctx.world > 1 else None
    f.close()

    alt = None
    if ctx.world > 1 and args.alt_modes == "auto":
        # the other coefficient mode split the same way (table: the C/C++/Fortran drop-in default; split counting,
        # run generation, group counts in the halo group), checked against the unsplit plane like the headline
        other = "table" if args.coeff_mode == "packed" else "packed"
        if ctx.rank == 0:
            progress(f"{name}: {other} mode over {ctx.world} rank(s)")
        saved_mode = args.coeff_mode
        args.coeff_mode = other
        try:
            h2, arec = run_config(dfamd, ctx, wl, args, ctx.comm_id(dfamd))
            asum = summarize(ctx, wl, args, ctx.gather(arec))
            aps = ctx.gather(parity_check(dfamd, ctx, wl, args, h2, h2.calls_done)) if args.parity == "on" else None
            acomm = h2.comm_info()
            h2.close()
        finally:
            args.coeff_mode = saved_mode
        ctx.barrier()
        alt = {other: {"value": asum["value"], "ms_per_step": asum["ms_per_step"],
                       "phase_ms_per_call": asum["phase_ms_per_call"], "multi_gpu": asum.get("multi_gpu"),
                       "parity_ok": all(p["ok"] for p in aps) if aps else None,
                       "rng_collective_bytes_per_call": acomm.get("rng_bytes_received")}}
    if ctx.world == 1 and args.alt_modes == "auto" and wl["plane"] != "native":
        other = "table" if args.coeff_mode == "packed" else "packed"
        g = make_filter(dfamd, ctx, wl, args, other)
        taps = sum(g.comp_info(c)["by_size"] + g.comp_info(c)["bz_size"] for c in range(3))
        # wall time without per-phase events (a 0.35 ms table-mode call feels the 6 event records per call),
        # then a second pass of K calls with them for the phase split and the FP64 roofline
        el2, _, _ = timed(ctx, g, args, min_warm_s=0.3, profile=False)
        el2p, p2, _ = timed(ctx, g, args)
        ms2 = el2 * 1e3 / args.steps
        cells = wl["Ny"] * wl["Nz"]
        alt = {other: {"value": round(cells * args.steps / el2, 1), "ms_per_step": round(ms2, 4),
                       "ms_per_step_with_phase_events": round(el2p * 1e3 / args.steps, 4),
                       "phase_ms_per_call": per_call(p2)}}
        if other == "table":
            alt[other]["note"] = ("same results bit for bit (parity below, tests/test_gpu_parity.py); coefficients "
                                  "read from a per-N table instead of the offset-packed stream, so SURVEY 8d's "
                                  "algorithmic bytes do not apply: FP64-VALU roofline below")
            # 2 flop (mul, add) per tap and cell (5.17 GFLOP at c3). Peak: MI355X FP64 vector
            # 78.6 TFLOP/s; the sums must not contract to FMA (bit-exactness), so mul+add caps at half.
            sw_ms = (p2["ypass_ms"] + p2["zpass_ms"]) / max(1, p2["calls"])
            flops = 2.0 * taps
            tf = flops / (sw_ms * 1e-3) / 1e12
            alt[other]["roofline_valu"] = {"bound": "valu-fp64", "achieved": round(tf, 2), "peak": 78.6,
                                           "unit": "TFLOP/s", "frac": round(tf / 78.6, 4),
                                           "flops_per_call": flops, "sweeps_ms": round(sw_ms, 4),
                                           "note": "mul+add without FMA contraction caps at 39.3 TFLOP/s"}
            vp = os.path.join(ROOT, "profiles", "r1", "probe", "valu_probe_fp64.jsonl")
            if os.path.exists(vp):  # measured FP64 mul+add issue ceiling (tools/valu_probe)
                best = max(json.loads(l)["wave_instr_per_s"] for l in open(vp) if l.startswith("{"))
                ceil_tf = best * 64 / 1e12
                alt[other]["roofline_valu"]["measured_ceiling"] = {
                    "TFLOPs": round(ceil_tf, 1), "frac": round(tf / ceil_tf, 4), "source": os.path.relpath(vp, ROOT)}
                # The whole call's VALU issue (sweeps AND the overlapped RNG) against the same ceiling: the
                # instruction count per call from a PMC pass (profiles/valu_issue.json), over this wall time.
                vi = os.path.join(ROOT, "profiles", "valu_issue.json")
                key = f"{name}/{other}"
                if os.path.exists(vi) and key in json.load(open(vi)).get("per_call_valu_wave_instr", {}):
                    n_instr = json.load(open(vi))["per_call_valu_wave_instr"][key]
                    rate = n_instr / (ms2 * 1e-3)
                    alt[other]["roofline_valu"]["call_issue"] = {
                        "valu_wave_instr_per_call": n_instr, "achieved_per_s": round(rate, 1),
                        "ceiling_per_s": best, "frac": round(rate / best, 4),
                        "source": os.path.relpath(vi, ROOT),
                        "note": "SQ_INSTS_VALU of every kernel of one call (sweeps + RNG) / wall ms_per_step, "
                                "against tools/valu_probe's FP64 issue ceiling"}
        g.close()

    ctx.barrier()
    same = None
    if ctx.world > 1 and args.same_plane == "auto":
        same = same_plane_1gpu(dfamd, ctx, wl, args, head["ms_per_step"])
    lr_steps = 0 if args.long_run == "auto" else int(args.long_run)
    lr = long_run(dfamd, ctx, wl, args, lr_steps, ctx.comm_id(dfamd)) if lr_steps > 0 else None

    others = {}
    for oname in filter(None, others_arg.split(",")):
        if oname == name or oname not in CONFIGS:
            continue
        try:
            owl = plan_workload(oname, ctx.world, args.scaling)
        except ValueError:
            continue
        if ctx.rank == 0:
            progress(f"{oname}: {owl['Ny']}x{owl['Nz']} over {ctx.world} rank(s)")
        h, orec = run_config(dfamd, ctx, owl, args, ctx.comm_id(dfamd), min_warm_s=0.3)
        orecs = ctx.gather(orec)
        osum = summarize(ctx, owl, args, orecs)
        op = ops = None
        if args.parity == "on":
            ops = ctx.gather(parity_check(dfamd, ctx, owl, args, h, h.calls_done))
            op = all(p["ok"] for p in ops)
        h.close()
        ctx.barrier()
        others[oname] = {"workload": owl["desc"], "Ny": owl["Ny"], "Nz": owl["Nz"], "scaling": owl["scaling"],
                         "parity_ok": op, **osum}
        if ops and not op:
            others[oname]["parity"] = [p for p in ops if not p["ok"]]
        if ctx.world > 1 and args.same_plane == "auto":
            others[oname]["same_plane_1gpu"] = same_plane_1gpu(dfamd, ctx, owl, args, osum["ms_per_step"])
        if oname == "c1" and ctx.world == 1 and ctx.rank == 0 and args.cpu_baseline == "auto":
            # BASELINE configs[0], the reference's CPU-runnable case: the reference itself on one core beside
            # the GPU's c1 line (test/cpp-main.cpp:12-17 builds this object; df.cpp:452-464 is its timer)
            try:
                rr = ref_time(args, owl["Ny"], owl["Nz"], owl["N_min"], owl["N_max"], 400, timeout=300)
                if rr is not None:
                    cells = owl["Ny"] * owl["Nz"]
                    others[oname]["cpu_reference"] = {
                        "value": round(cells / rr["mean_s"], 1), "unit": "cells/s", "cores": 1, "kind": "reference",
                        "ms_per_call": round(rr["mean_s"] * 1e3, 4), "calls": 400,
                        "gpu_over_cpu": round(osum["value"] / (cells / rr["mean_s"]), 1)}
            except Exception as e:
                others[oname]["cpu_reference"] = {"error": str(e)[-300:]}
        if oname == "c5" and ctx.world > 1 and args.long_run == "auto":
            others[oname]["long_run"] = long_run(dfamd, ctx, owl, args, 10000, ctx.comm_id(dfamd))

    if ctx.world == 1 and "native" in others and args.alt_modes == "auto" and args.coeff_mode == "packed":
        # the reference's own grid in table mode - the C/C++/Fortran drop-in default on the only plane the
        # reference computes - with its FP64 roofline, as alt_modes.table for c3
        owl = plan_workload("native", ctx.world, args.scaling)
        g = make_filter(dfamd, ctx, owl, args, "table")
        taps = sum(g.comp_info(c)["by_size"] + g.comp_info(c)["bz_size"] for c in range(3))
        el2, _, n2 = timed(ctx, g, args, min_warm_s=0.3, profile=False, label="native table")
        el2p, p2, n3 = timed(ctx, g, args, label="native table, phase events")
        ms2 = el2 * 1e3 / args.steps
        cells = owl["Ny"] * owl["Nz"]
        sw_ms = (p2["ypass_ms"] + p2["zpass_ms"]) / max(1, p2["calls"])
        tf = 2.0 * taps / (sw_ms * 1e-3) / 1e12
        nt = {"workload": owl["desc"] + ", table mode", "Ny": owl["Ny"], "Nz": owl["Nz"],
              "value": round(cells * args.steps / el2, 1), "ms_per_step": round(ms2, 4),
              "ms_per_step_with_phase_events": round(el2p * 1e3 / args.steps, 4), "phase_ms_per_call": per_call(p2),
              "launch_shape": {k: g.get_tuning(k) for k in ("ylds", "yt_rows", "yt_chunk", "handoff_batch", "gen_dense")},
              "roofline_valu": {"bound": "valu-fp64", "achieved": round(tf, 2), "peak": 78.6, "unit": "TFLOP/s",
                                "frac": round(tf / 78.6, 4), "flops_per_call": 2.0 * taps, "sweeps_ms": round(sw_ms, 4),
                                "note": "2 flop per tap and cell over the y- and z-pass phase time (hipEvents; the "
                                        "RNG of later calls runs beside them); mul+add without FMA caps at 39.3"}}
        vp = os.path.join(ROOT, "profiles", "r1", "probe", "valu_probe_fp64.jsonl")
        if os.path.exists(vp):
            best = max(json.loads(l)["wave_instr_per_s"] for l in open(vp) if l.startswith("{"))
            nt["roofline_valu"]["measured_ceiling"] = {"TFLOPs": round(best * 64 / 1e12, 1),
                                                       "frac": round(tf / (best * 64 / 1e12), 4),
                                                       "source": os.path.relpath(vp, ROOT)}
        if args.parity == "on":
            ops = ctx.gather(parity_check(dfamd, ctx, owl, args, g, n2 + n3))
            nt["parity_ok"] = all(p["ok"] for p in ops)
        g.close()
        others["native_table"] = nt

    dropin = None
    rank_phase("reports (drop-in, CPU baseline, JSON line)")
    if ctx.rank == 0 and ctx.world == 1 and args.dropin == "auto":
        dropin = dropin_timing(args)
        nd = dropin.get("native/table", {})
        if "native_table" in others and "capi_ms" in nd:
            # the drop-in default's per-step cost on the reference's grid, beside its async figure:
            # df_filter + df_wait (this call's fields only), + df_sync (later calls' noise too), and the C++ filter()
            others["native_table"]["synchronous_call"] = {
                "capi_ms": nd["capi_ms"], "capi_sync_all_ms": nd.get("capi_sync_all_ms"),
                "dropin_mirror0_ms": nd["dropin_ms"]["mirror0"],
                "dropin_stream_ordered_ms": nd["dropin_ms"].get("mirror0_stream_ordered"),
                "ypass_ahead": nd.get("ypass_ahead"), "capi_ms_ypass_ahead_flipped": nd.get("capi_ms_ypass_ahead_flipped"),
                "note": "examples/cpp-test time, 60 calls each: a synchronous caller's wall per step"}
    if ctx.rank == 0:
        cpu = cpu_par = None
        if args.cpu_baseline == "auto" and ctx.world == 1 and wl["plane"] != "native":
            try:
                cpu = cpu_baseline(args, wl["Ny"], wl["Nz"], wl["N_min"], wl["N_max"])
            except Exception as e:  # reported, never fatal for the GPU number
                cpu = {"error": str(e)}
            try:
                cpu_par = cpu_baseline_parallel(args, wl["Ny"], wl["N_min"], wl["N_max"])
            except Exception as e:
                cpu_par = {"error": str(e)}
        ms = head["ms_per_step"]
        call_bytes = sum(r["call_bytes"] for r in recs)  # SURVEY 8d algorithmic bytes of one call, all ranks
        out = {
            "metric": "inflow cells/sec (filter(dt) call) + achieved HBM GB/s, 1/2/4/8 GPU",
            "value": head["value"],
            "unit": "cells/s",
            "n_gpus": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": wl["scaling"],
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY 8d plane; rows from files/RST.dat + line.dat; pcg32 seed %d)" % args.seed,
            "config": {"workload": wl["desc"], "name": name, "Ny": wl["Ny"], "Nz": wl["Nz"], "N_min": wl["N_min"],
                       "N_max": wl["N_max"], "dt": args.dt, "coeff_mode": args.coeff_mode,
                       "rows_per_wave": args.rows_per_wave,
                       "parallelism": f"z-strips x{ctx.world}" if ctx.world > 1 else "single GPU"},
            "emulated_hosts": ctx.emulated or None,
            "parity_ok": parity["ok"] if parity else None,
            "rng_collective": RNG_COLLECTIVE.get((comm or {}).get("rng_collective", 0), "?").split(":")[0],
            "phase_ms_per_call": head["phase_ms_per_call"],
            "roofline": head["roofline"],
            "cpu_baseline": cpu,
            "cpu_baseline_parallel": cpu_par,
            "alt_modes": alt,
            "other_configs": others or None,
            "parity": parity,
            "setup_s": rec["setup_s"],
        }
        out["achieved_call_GBps"] = round(call_bytes / (ms * 1e-3) / 1e9, 1)
        out["call_hbm_frac"] = round(call_bytes / (ms * 1e-3) / 1e9 / (HBM_PEAK_GBPS * ctx.world), 4)
        if "multi_gpu" in head:
            out["multi_gpu"] = head["multi_gpu"]
        if same is not None:
            out["ms_per_step_1gpu_same_plane"] = same["ms_per_step"]
            out["speedup"] = same["speedup"]
            out["same_plane_1gpu"] = same
        if lr is not None:
            out["long_run"] = lr
        if dropin is not None:
            out["dropin"] = dropin
        print(json.dumps(out), flush=True)
    ctx.barrier()
    if ctx.dist is not None:
        ctx.dist.destroy_process_group()
    rank_phase("done")
    return 0


if __name__ == "__main__":
    try:
        sys.exit(main())
    except Exception as e:  # the rank's last phase names the failure for the launching parent
        rank_phase(f"failed: {type(e).__name__}: {str(e)[:200]}")
        raise
