#!/bin/bash
# Table-mode y-pass shapes on c3 (rows per wave 4 vs 8 vs 2, with the RNG overlapped and alone).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2q
mkdir -p $O
for t in "rows_per_wave=4 rows_per_wave=8" "rows_per_wave=4 rows_per_wave=2" "rows_per_wave=4,ywindow=1 rows_per_wave=4,ywindow=0"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a $1 --tune-b $2 --config c3 --mode table --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
timeout -k 10 300 python tools/ab.py --tune-a rows_per_wave=4 --tune-b rows_per_wave=8 --config c3 --mode table --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], d['A'], d['A_median_ms'], d['B'], d['B_median_ms'])"
