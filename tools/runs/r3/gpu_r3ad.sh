#!/bin/bash
# c3 table, RNG overlap off: kernel timeline of one call (every RNG kernel and the gaps between them).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ad; mkdir -p $O
DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
   python3 $R/tools/ab.py --config c3 --mode table --rounds 3 --calls 10 > $O/ab.json 2> $O/prof.err || { echo "rocprof failed"; tail -5 $O/prof.err; exit 1; }
python3 $R/tools/rocprof_split.py $O/prof/run_kernel_trace.csv > $O/kernel_split.csv
head -20 $O/kernel_split.csv
python3 - <<'PY' > $O/timeline.txt
import csv
rows = list(csv.DictReader(open("/root/repo/gpurun_out/r3ad/prof/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-40:]
t0 = int(rows[0]["Start_Timestamp"])
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0
    prev = e
    print(f'{(s-t0)/1e3:10.2f} {(e-t0)/1e3:10.2f} dur {(e-s)/1e3:8.2f} gap {gap:7.2f} {r["Kernel_Name"][:70]}')
PY
cat $O/timeline.txt
rm -f $O/prof/run_kernel_trace.csv
