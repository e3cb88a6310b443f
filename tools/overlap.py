#!/usr/bin/env python3
"""How much of each sweep kernel's time runs beside the noise generation, from a rocprofv3 kernel trace.

For every y-pass and z-pass launch (after the first `skip` calls), the share of its duration during which
at least one rng_* kernel was running, and the mean duration with and without such overlap.
    python3 tools/overlap.py <dir>/run_kernel_trace.csv [skip]"""
import csv
import sys


def merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(s, e, rng):
    t = 0
    for a, b in rng:  # rng is merged and sorted; planes here have a few thousand intervals
        if b <= s:
            continue
        if a >= e:
            break
        t += min(b, e) - max(a, s)
    return t


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    iv = lambda r: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    rng = merge([iv(r) for r in rows if "rng_" in r["Kernel_Name"]])
    for kind in ("ypass", "zpass"):
        ks = [iv(r) for r in rows if kind in r["Kernel_Name"]][skip:]
        if not ks:
            continue
        dur = [e - s for s, e in ks]
        cov = [covered(s, e, rng) for s, e in ks]
        frac = sum(cov) / sum(dur)
        alone = [d for d, c in zip(dur, cov) if c < 0.05 * d]
        beside = [d for d, c in zip(dur, cov) if c >= 0.5 * d]
        mean = lambda v: sum(v) / len(v) / 1e3 if v else float("nan")
        print(f"{kind}: {len(ks)} launches, mean {mean(dur):.1f} us, {100 * frac:.0f}% of their time beside rng_*; "
              f"mean alone {mean(alone):.1f} us ({len(alone)}), beside >= half {mean(beside):.1f} us ({len(beside)})")


if __name__ == "__main__":
    main()
