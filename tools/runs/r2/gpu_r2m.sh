#!/bin/bash
# Does loading torch first (as bench.py does) change the table-mode sweeps? Same A/B, with and without.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2m
mkdir -p $O
timeout -k 10 300 python tools/ab.py --tune-a gen_compact=1 --tune-b gen_compact=1 --config c3 --mode table --rounds 5 --calls 20 > $O/ab_notorch.json 2> $O/err \
  || { echo "ab failed"; tail -20 $O/err; exit 1; }
timeout -k 10 300 python tools/ab.py --torch --tune-a gen_compact=1 --tune-b gen_compact=1 --config c3 --mode table --rounds 5 --calls 20 > $O/ab_torch.json 2>> $O/err \
  || { echo "ab failed"; tail -20 $O/err; exit 1; }
python3 -c "
import json
for f in ('ab_notorch', 'ab_torch'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['A_median_ms'])"
