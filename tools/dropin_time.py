#!/usr/bin/env python3
"""The drop-in's per-call cost alone (bench.py `dropin`, examples/cpp-test `time`): one JSON line per plane and
mode, `--repeat` times, without the rest of the bench.

    python3 tools/dropin_time.py [--repeat 3] [--calls 60] [--planes native,c3]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "cpp-test")
DIMS = {"native": ("native", "0", "0", "0", "0"), "c3": ("synth", "2048", "2048", "4", "64"),
        "c2": ("synth", "512", "512", "4", "32")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--calls", type=int, default=60)
    ap.add_argument("--planes", default="native,c3")
    ap.add_argument("--modes", default="table,packed")
    a = ap.parse_args()
    for rep in range(a.repeat):
        for plane in a.planes.split(","):
            for mode in a.modes.split(","):
                r = subprocess.run([EXE, "time", *DIMS[plane], mode, str(a.calls)], capture_output=True, text=True,
                                   timeout=300, check=True)
                rec = json.loads(r.stdout.strip().splitlines()[-1])
                rec.update(repeat=rep, config=plane)
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    sys.exit(main())
