#!/bin/bash
# Row-pair y-pass: per-tile cost in the XCD balance (ycoop_ovh) for ycoop 7 / 8 on the reference's grid.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2w}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "native_grid or runtime_tuning" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for t in "ycoop=7 ycoop=11" "ycoop=7 ycoop=12" "ycoop=4 ycoop=7" "ycoop=7 ycoop=10"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a $1 --tune-b $2 --config native --mode packed --rounds 9 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], d['A'], d['A_median_ms']['ypass_ms'], d['A_median_ms']['wall_ms'], d['B'], d['B_median_ms']['ypass_ms'], d['B_median_ms']['wall_ms'])"
