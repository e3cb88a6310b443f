#!/bin/bash
# Cooperative y-pass (ycoop) parity + A/B, and write windows with a co-tenant (tools/cotenant.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "native packed" "c2 packed" "c3 packed"; do
  set -- $cfg
  timeout -k 10 300 python tools/ab.py --tune-a ycoop=0 --tune-b ycoop=1 --config $1 --mode $2 --rounds 7 --calls 20 >> $O/ab_ycoop.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab_ycoop.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], 'A', d['A_median_ms'], 'B', d['B_median_ms'])"
timeout -k 10 300 python tools/cotenant.py --config c3 --mode packed --rounds 5 --calls 30 > $O/cotenant_c3.json 2> $O/cotenant.err \
  || { echo "cotenant failed"; tail -20 $O/cotenant.err; exit 1; }
cat $O/cotenant_c3.json
