#!/usr/bin/env python3
"""Per-(kernel, grid) summary of a rocprofv3 kernel trace.

bench.py's default run times c3 and then, in the same process, the table mode and the other
configs (the reference's grid, c2); rocprofv3's --stats averages every launch of a kernel name
together, whatever its grid. This splits run_kernel_trace.csv by launch grid so the c3 launches of
the dominant kernel can be read against bench.py's roofline.avg_launch_ms.

    python3 tools/rocprof_split.py <dir>/run_kernel_trace.csv [> split.csv]
"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    rows = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        grid = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        rows[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid_x", "grid_y", "grid_z", "calls", "avg_us", "median_us", "min_us", "max_us", "total_us"])
    for (name, grid), d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, *grid, len(d), round(statistics.mean(d), 2), round(statistics.median(d), 2),
                    round(min(d), 2), round(max(d), 2), round(sum(d), 1)])


if __name__ == "__main__":
    main()
