#!/bin/bash
# Small planes: the compacted K3 plans its own waves (fuse_plan) instead of a scan-and-plan launch:
# parity, then A/B on the small planes (host-bound table mode, device-bound packed).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2ak}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cm in "c2 table" "native table" "c1 table" "c1 packed" "c2 packed" "native packed"; do
  set -- $cm
  timeout -k 10 300 python tools/ab.py --tune-a fuse_plan=0 --tune-b fuse_plan=1 --config $1 --mode $2 --rounds 9 --calls 40 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); a=d['A_median_ms']; b=d['B_median_ms']; print(d['config'], d['mode'], d['A'], a.get('rng_ms'), a['wall_ms'], '|', d['B'], b.get('rng_ms'), b['wall_ms'])"
