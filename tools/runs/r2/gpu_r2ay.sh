#!/bin/bash
# The reference's grid, packed: y-pass forms re-checked with the pooled coefficient allocation.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2ay}
mkdir -p $O
for t in "ycoop=7 ycoop=8" "ycoop=7 ycoop=4" "ycoop=7 ycoop=0" "ycoop=7 ycoop=3"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --tune-a $1 --tune-b $2 --config native --mode packed --rounds 9 --calls 40 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); a=d['A_median_ms']; b=d['B_median_ms']; print(d['config'], d['mode'], d['A'], a.get('ypass_ms'), a['wall_ms'], '|', d['B'], b.get('ypass_ms'), b['wall_ms'])"
