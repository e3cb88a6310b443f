#!/bin/bash
# Coefficient arrays pooled in one allocation (DFAMD_B_POOL 1: per component, 2: per direction) against
# one allocation each: 4 c3 packed handles per setting, alive at once; a parity check with each pooled form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2au}
mkdir -p $O
for pl in 1; do
  DFAMD_B_POOL=$pl timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "bitexact or golden" > $O/pytest_$pl.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest_$pl.log; exit 1; }
  tail -1 $O/pytest_$pl.log
done
for pl in 0 1 0 1 2; do
  DFAMD_B_POOL=$pl timeout -k 10 300 python tools/handle_var.py 4 >> $O/pool_$pl.jsonl 2> $O/pool_$pl.err || { echo "failed"; tail -20 $O/pool_$pl.err; exit 1; }
done
python3 -c "
import json, statistics
for pl in (0, 1, 2):
    d=[json.loads(l) for l in open('$O/pool_%d.jsonl' % pl)]
    print('pool', pl, 'mean total', round(statistics.mean(x['total_ms'] for x in d),4), 'min', min(x['total_ms'] for x in d), 'max', max(x['total_ms'] for x in d), 'n', len(d))"
