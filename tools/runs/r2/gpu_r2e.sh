#!/bin/bash
# Native-grid y-pass with the RNG overlap off: per-wave vs cooperative, and rows/unroll shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2e
mkdir -p $O
for t in "ycoop=0 ycoop=1" "ycoop=0,rows_per_wave=1,yunroll=8 ycoop=0,rows_per_wave=2,yunroll=8" "ycoop=0,rows_per_wave=1,yunroll=4 ycoop=0,rows_per_wave=1,yunroll=2"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a $1 --tune-b $2 --config native --mode packed --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a ycoop=0 --tune-b ycoop=1 --config native --mode table --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], d['A'], d['A_median_ms'], d['B'], d['B_median_ms'])"
