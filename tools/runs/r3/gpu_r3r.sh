#!/bin/bash
# Reference's grid, packed: is the call bound by the y-pass or by the next call's RNG beside it?
# RNG overlap on vs off (main and no-load ablation libraries), and a rocprofv3 kernel trace of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3r
mkdir -p $O
L=$GRAFT_REPO_ROOT/digital-filtering_amd
for v in "" _nocoefnoise; do
  DFAMD_LIB=$L/libdfamd$v.so timeout -k 10 120 python3 tools/ab.py --config native --mode packed --rounds 9 --calls 20 \
    --a DFAMD_RNG_OVERLAP=0 --b DFAMD_RNG_OVERLAP=1 > $O/ab_overlap$v.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_overlap$v.json'));print('lib$v overlap0', d['A_median_ms'], 'overlap1', d['B_median_ms'])"
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
   python3 $GRAFT_REPO_ROOT/tools/ab.py --config native --mode packed --rounds 5 --calls 20 > $O/ab_prof.json 2> $O/prof.err) \
   || { echo "rocprof failed"; tail -5 $O/prof.err; exit 1; }
python3 tools/rocprof_split.py $O/prof/run_kernel_trace.csv > $O/kernel_split.csv
cat $O/kernel_split.csv
python3 - <<'PY' > $O/timeline.txt
import csv
rows = list(csv.DictReader(open("/root/repo/gpurun_out/r3r/prof/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[-200]["Start_Timestamp"])
for r in rows[-200:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{(s-t0)/1e3:10.2f} {(e-t0)/1e3:10.2f} {(e-s)/1e3:8.2f} q{r.get("Queue_Id","")} {r["Kernel_Name"][:60]}')
PY
head -60 $O/timeline.txt
rm -f $O/prof/run_kernel_trace.csv
