#!/bin/bash
# Table z-pass with four cells per lane (zquad): parity, then A/B per config (table mode).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2ad}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "zquad or runtime_tuning or lds_staging or table_mode" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a zquad=0 --tune-b zquad=1 --config c3 --mode table --rounds 9 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
  || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
for cfg in c3 native c2; do
  timeout -k 10 300 python tools/ab.py --tune-a zquad=0 --tune-b zquad=1 --config $cfg --mode table --rounds 9 --calls 40 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); a=d['A_median_ms']; b=d['B_median_ms']; print(d['config'], d['mode'], d['A'], a.get('zpass_ms'), a['wall_ms'], '|', d['B'], b.get('zpass_ms'), b['wall_ms'])"
