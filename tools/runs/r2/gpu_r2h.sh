#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2h
mkdir -p $O
for t in "ycoop=0,nt_loads=1 ycoop=0,nt_loads=0" "ycoop=1,heavy_first=0 ycoop=2,heavy_first=0" "ycoop=0,heavy_first=0 ycoop=1,heavy_first=0" "ycoop=1,heavy_first=0,nt_loads=0 ycoop=1,heavy_first=1,nt_loads=0"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a $1 --tune-b $2 --config native --mode packed --rounds 9 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
timeout -k 10 300 python tools/ab.py --tune-a ycoop=0,heavy_first=1 --tune-b ycoop=1,heavy_first=0 --config native --mode packed --rounds 9 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], d['A'], d['A_median_ms']['ypass_ms'], d['A_median_ms']['wall_ms'], d['B'], d['B_median_ms']['ypass_ms'], d['B_median_ms']['wall_ms'])"
