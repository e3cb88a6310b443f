#!/bin/bash
# fuse_plan on packed planes without long y chains (c1, c2): parity, then A/B against the scan-and-plan launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2ao}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cm in "c2 packed" "c1 packed" "c2 packed" "native packed"; do
  set -- $cm
  timeout -k 10 300 python tools/ab.py --tune-a fuse_plan=0 --tune-b fuse_plan=1 --config $1 --mode $2 --rounds 11 --calls 40 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); a=d['A_median_ms']; b=d['B_median_ms']; print(d['config'], d['mode'], d['A'], a.get('rng_ms'), a['wall_ms'], '|', d['B'], b.get('rng_ms'), b['wall_ms'])"
