#!/bin/bash
# One rank of an 8-way c4 split, packed, with and without the pooled coefficient allocation.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2az}
mkdir -p $O
for pl in 1 0 1 0; do
  DFAMD_B_POOL=$pl timeout -k 10 300 python tools/strip_timing.py --config c4 --mode packed --replicate 1 --ns 8,1 --tune "" >> $O/strip_pool$pl.jsonl 2>> $O/strip.err \
    || { echo "strip failed"; tail -20 $O/strip.err; exit 1; }
done
python3 -c "
import json
for pl in (1, 0):
    for l in open('$O/strip_pool%d.jsonl' % pl):
        d=json.loads(l); print('pool', pl, 'N', d['N'], 'rank', d['rank'], 'wall', d['wall_ms'], 'y', d['ypass_ms'], 'z', d['zpass_ms'])"
