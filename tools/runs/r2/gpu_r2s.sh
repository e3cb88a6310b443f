#!/bin/bash
# Component-split packed z-pass (zsplit): parity, then A/B on c2, the native grid, c1 and c3 (packed).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2s
mkdir -p $O
rm -f $O/ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "tuning or golden or strips" --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in c2 native c1 c3; do
  timeout -k 10 300 python tools/ab.py --tune-a zsplit=0 --tune-b zsplit=1 --config $cfg --mode packed --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], d['A'], d['A_median_ms'], d['B'], d['B_median_ms'])"
