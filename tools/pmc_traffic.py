#!/usr/bin/env python3
"""Measure real HBM traffic per launch of the hot kernels with rocprofv3 PMC
counters, calibrated as MI355X_MICROARCH.md §HBM prescribes.

Runs (on the GPU box), each counter in its own pass, counters only:
  rocprofv3 --pmc FETCH_SIZE  -- tools/hbm_probe pmc          (known 1 GiB reads/writes)
  rocprofv3 --pmc WRITE_SIZE  -- tools/hbm_probe pmc
  rocprofv3 --pmc FETCH_SIZE  -- python3 bench.py ... (per coeff mode)
  rocprofv3 --pmc WRITE_SIZE  -- python3 bench.py ...
FETCH_SIZE/WRITE_SIZE are KiB. On gfx950 FETCH_SIZE reads 1/2 of a wide
coalesced stream; the probe's known byte counts give the read and write
factors for the access widths the kernels use (16-B loads; 8-B and 16-B stores).
Writes profiles/pmc_traffic.json, which bench.py reports as roofline.traffic.
"""
import argparse
import csv
import glob
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pmc(counter, outdir, cmd, timeout=600):
    os.makedirs(outdir, exist_ok=True)
    full = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", outdir, "-o", "run", "--"] + cmd
    subprocess.run(["timeout", "-k", "10", str(timeout)] + full, check=True, cwd="/tmp",
                   stdout=open(os.path.join(outdir, "stdout.log"), "w"), stderr=subprocess.STDOUT)


def parse(outdir, counter):
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise RuntimeError(f"no counter_collection.csv under {outdir}")
    per = {}
    for row in csv.DictReader(open(files[0])):
        if row.get("Counter_Name") != counter:
            continue
        name = row.get("Kernel_Name", "")
        per.setdefault(name, []).append(float(row["Counter_Value"]))
    return per


def short(name):
    for k in ("ypass", "zpass"):  # every y-pass form (packed, coop2, table, t64, tlds) is the launch's y-pass
        if k + "_" in name:
            return k + "_kernel"
    for k in ("ypass_kernel", "zpass_kernel", "rng_generate_kernel", "rng_count_kernel", "expand_coeffs_kernel",
              "read_kernel<false>", "read_kernel<true>", "write_kernel<1>", "write_kernel<2>"):
        if k in name:
            return k
    return name[:60]


def collapse(per):
    out = {}
    for name, vals in per.items():
        out.setdefault(short(name), []).extend(vals)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    ap.add_argument("--configs", default="c3:packed+table,c2:packed,native:packed,c1:packed",
                    help="config:mode+mode,... (the N = 1 bench line's planes)")
    ap.add_argument("--json", default=os.path.join(ROOT, "gpurun_out", "pmc_traffic.json"))  # copy to profiles/
    a = ap.parse_args()
    a.out, a.json = os.path.abspath(a.out), os.path.abspath(a.json)  # rocprofv3 runs from /tmp
    probe = [os.path.join(ROOT, "tools", "hbm_probe"), "pmc"]
    plan = [(c.split(":")[0], m) for c in a.configs.split(",") for m in c.split(":")[1].split("+")]
    res = {"method": __doc__.strip().splitlines()[0], "configs": a.configs, "raw_kib": {}, "per_launch_bytes": {}}
    raw = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(a.out, f"probe_{counter}")
        run_pmc(counter, d, probe)
        raw[("probe", counter)] = collapse(parse(d, counter))
        for cfg, mode in plan:
            d = os.path.join(a.out, f"{cfg}_{mode}_{counter}")
            run_pmc(counter, d, [sys.executable, os.path.join(ROOT, "bench.py"), "--config", cfg,
                                 "--coeff-mode", mode, "--steps", "3", "--warmup", "1", "--cpu-baseline", "off",
                                 "--alt-modes", "off", "--other-configs", "", "--parity", "off"])
            raw[(cfg, mode, counter)] = collapse(parse(d, counter))
    gib = float(1 << 30)
    raw = {(k[0], k[1]) if k[0] == "probe" else k: v for k, v in raw.items()}
    pf = raw[("probe", "FETCH_SIZE")]
    pw = raw[("probe", "WRITE_SIZE")]
    cal = {
        "read16_factor": gib / (statistics.median(pf["read_kernel<false>"]) * 1024),
        "read16_nt_factor": gib / (statistics.median(pf["read_kernel<true>"]) * 1024),
        "write8_factor": gib / (statistics.median(pw["write_kernel<1>"]) * 1024),
        "write16_factor": gib / (statistics.median(pw["write_kernel<2>"]) * 1024),
    }
    res["calibration"] = cal
    for cfg, mode in plan:
        f = raw[(cfg, mode, "FETCH_SIZE")]
        w = raw[(cfg, mode, "WRITE_SIZE")]
        for k, wfac in (("ypass_kernel", cal["write16_factor"]), ("zpass_kernel", cal["write8_factor"])):
            if k not in f or k not in w:
                continue
            fk = statistics.median(f[k][1:] if len(f[k]) > 1 else f[k])  # skip the constructor's step 0
            wk = statistics.median(w[k][1:] if len(w[k]) > 1 else w[k])
            rfac = cal["read16_nt_factor"] if mode == "packed" else cal["read16_factor"]
            key = f"{cfg}/{mode}/{k.split('_')[0]}"
            res["per_launch_bytes"][key] = fk * 1024 * rfac + wk * 1024 * wfac
            res["raw_kib"][key] = {"FETCH_SIZE": fk, "WRITE_SIZE": wk}
        for k in ("rng_generate_kernel", "rng_count_kernel"):
            if k in f and k in w:
                res["raw_kib"][f"{cfg}/{mode}/{k}"] = {"FETCH_SIZE": statistics.median(f[k]),
                                                           "WRITE_SIZE": statistics.median(w[k])}
    res["raw_kib"]["probe"] = {f"{key[1]}:{k}": statistics.median(v) for key, d in raw.items() if key[0] == "probe"
                               for k, v in d.items()}
    os.makedirs(os.path.dirname(a.json), exist_ok=True)
    json.dump(res, open(a.json, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
