#!/bin/bash
# Wave-tile y-pass with XCD runs of equal bytes (ybalance): parity, then A/B per config and mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2ac}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cm in "c2 packed" "c2 table" "c3 packed" "c3 table" "native table" "c1 packed"; do
  set -- $cm
  timeout -k 10 300 python tools/ab.py --tune-a ybalance=0 --tune-b ybalance=1 --config $1 --mode $2 --rounds 9 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); a=d['A_median_ms']; b=d['B_median_ms']; print(d['config'], d['mode'], d['A'], a['ypass_ms'], a['wall_ms'], '|', d['B'], b['ypass_ms'], b['wall_ms'])"
