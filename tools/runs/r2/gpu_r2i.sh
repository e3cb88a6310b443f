#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2i
mkdir -p $O
for t in "ycoop=2 ycoop=3" "ycoop=0 ycoop=2" "ycoop=1 ycoop=3"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a $1 --tune-b $2 --config native --mode packed --rounds 9 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
for t in "ycoop=0 ycoop=2" "ycoop=0 ycoop=3"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --tune-a $1 --tune-b $2 --config native --mode packed --rounds 9 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], d['A'], d['A_median_ms']['ypass_ms'], d['A_median_ms']['wall_ms'], d['B'], d['B_median_ms']['ypass_ms'], d['B_median_ms']['wall_ms'])"
