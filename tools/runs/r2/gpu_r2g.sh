#!/bin/bash
# Native-grid y-pass with rows launched by falling half-width: per-wave vs cooperative (16 / 8 taps per wave).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "native or tuning or grid" --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for t in "ycoop=0 ycoop=1" "ycoop=0 ycoop=2" "ycoop=0,heavy_first=0 ycoop=1,heavy_first=0"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a $1 --tune-b $2 --config native --mode packed --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
for t in "ycoop=0 ycoop=1"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --tune-a $1 --tune-b $2 --config native --mode packed --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err
  timeout -k 10 300 python tools/ab.py --tune-a rows_per_wave=2 --tune-b rows_per_wave=1 --config native --mode table --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], d['A'], d['A_median_ms'], d['B'], d['B_median_ms'])"
