#!/bin/bash
# Kernel timelines without phase events (tools/plane_loop.py): c2 packed, the reference's grid packed and table,
# c3 table - the gaps between a call's kernels and between calls.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3aj; mkdir -p $O
for cm in "c2 packed" "native packed" "native table" "c3 table"; do
  set -- $cm
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$1_$2 -o run -- \
     python3 $R/tools/plane_loop.py $1 $2 60 > $O/$1_$2.log 2>&1 || { echo "rocprof $1 $2 failed"; tail -5 $O/$1_$2.log; exit 1; }
  python3 - $O/$1_$2/run_kernel_trace.csv > $O/timeline_$1_$2.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"]][-40:]
t0 = int(rows[0]["Start_Timestamp"])
ends = {}
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{(s-t0)/1e3:9.2f} {(e-t0)/1e3:9.2f} dur {(e-s)/1e3:7.2f}  {r["Kernel_Name"][:70]}')
PY
  echo "== $1 $2"; tail -14 $O/timeline_$1_$2.txt
  rm -f $O/$1_$2/run_kernel_trace.csv
done
