"""Bit-for-bit check of ypass_t64 forms against the default handle on the reference's grid (table mode).

Timing-only forms selected by DFAMD_YT_DEBUG (read when a handle is created) are compared with a handle made
without it; the default handle itself is checked against the oracle by tests/test_gpu_parity.py.
    python tools/t64_cmp.py DEBUG yt_rows=1 yt_rows=2 ...
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "digital-filtering_amd"))
import dfamd  # noqa: E402

FIELDS = ("u", "v", "w")


def run(tuning, debug):
    os.environ["DFAMD_YT_DEBUG"] = str(debug)
    g = dfamd.DigitalFilter(seed=42, device=0, coeff_mode="table")
    os.environ.pop("DFAMD_YT_DEBUG")
    g.set_tuning("ylds", 3)
    for k, v in tuning.items():
        g.set_tuning(k, v)
    out = []
    for dt in (None, 1e-8, 1e-5):
        if dt is not None:
            g.filter(dt)
        f = g.fields()
        out.append({k: np.array(f[k]) for k in FIELDS})
    g.close()
    return out


def main():
    debug = int(sys.argv[1])
    ref = run({}, 0)
    bad = 0
    for spec in sys.argv[2:]:
        tuning = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in spec.split(",")}
        got = run(tuning, debug)
        same = all(np.array_equal(a[k], b[k]) for a, b in zip(got, ref) for k in FIELDS)
        print(f"t64_cmp debug={debug} {spec}: {'identical' if same else 'DIFFERENT'}", flush=True)
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
