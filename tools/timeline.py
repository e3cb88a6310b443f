#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 kernel trace: the last `n` kernels in start order, with start and end in
microseconds from the first of them, queue (stream) and duration - to see what overlaps what.
    python3 tools/timeline.py <dir>/run_kernel_trace.csv [n]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dfamd::", "")[:48]
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        q = r.get("Queue_Id") or r.get("Stream_Id") or ""
        print(f"{s / 1e3:10.1f} {e / 1e3:10.1f} {(e - s) / 1e3:8.1f}  q{q:>3} {name} grid={r['Grid_Size_X']}")


if __name__ == "__main__":
    main()
