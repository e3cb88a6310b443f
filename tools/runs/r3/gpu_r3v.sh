#!/bin/bash
# HBM read bytes (FETCH_SIZE, x2 for 16-B streams on gfx950) of the row-pair y-pass on the reference's grid,
# XCD runs vs interleaved tiles, RNG overlap off; and plain vs non-temporal coefficient loads timed.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3v; mkdir -p $O
for m in 0 1; do
  DFAMD_RNG_OVERLAP=0 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/f$m -o run --output-format csv -- \
    python3 $R/tools/ab.py --config native --mode packed --rounds 2 --calls 5 --tune-a ycoop_map=$m --tune-b ycoop_map=$m > $O/f$m.log 2>&1
  rc=$?; echo "map $m FETCH_SIZE rc=$rc"; [ $rc = 0 ] || exit 1
  python3 - $O/f$m <<'PY'
import csv, glob, sys, statistics
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if "coop2" in r["Kernel_Name"]]
print("coop2 dispatches", len(v), "FETCH_SIZE KiB median", statistics.median(v), "-> GB x2:", 2 * statistics.median(v) * 1024 / 1e9)
PY
done
cd $R
for t in "ycoop_map=0" "ycoop_map=1"; do
  DFAMD_RNG_OVERLAP=0 timeout -k 10 120 python3 tools/ab.py --config native --mode packed --rounds 9 --calls 20 \
    --tune-a $t,nt_loads=1 --tune-b $t,nt_loads=0 > $O/ab_nt_$t.json || exit 1
  python3 -c "import json;d=json.load(open('$O/ab_nt_$t.json'));print('$t nt1', d['A_median_ms']['ypass_ms'], 'nt0', d['B_median_ms']['ypass_ms'])"
done
