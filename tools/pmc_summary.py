#!/usr/bin/env python3
"""Per-kernel means of the PMC passes written by tools/pmc_sweeps.sh / pmc_rng.sh.

    python3 tools/pmc_summary.py gpurun_out/pmcsw_table [kernel-substring ...]

Prints one JSON object: {kernel: {counter: mean per dispatch, ..., "dispatches": n}} plus
derived ratios where the counters are present (VALU busy = SQ_ACTIVE_INST_VALU * 4 /
(SQ_BUSY_CU_CYCLES * ... ) is left to the reader; the raw means are what is recorded)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    keys = sys.argv[2:] or ["ypass", "zpass"]
    sums = defaultdict(lambda: defaultdict(float))
    counts = defaultdict(lambda: defaultdict(set))
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            k = next((k for k in keys if k in name), None)
            if k is None:
                continue
            short = name.split("(")[0].replace("void dfamd::", "")
            c = row["Counter_Name"]
            sums[short][c] += float(row["Counter_Value"])
            counts[short][c].add((f, row.get("Dispatch_Id", row.get("Correlation_Id"))))
    out = {}
    for kern, cs in sums.items():
        out[kern] = {c: v / max(1, len(counts[kern][c])) for c, v in sorted(cs.items())}
        out[kern]["dispatches"] = max(len(s) for s in counts[kern].values())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
