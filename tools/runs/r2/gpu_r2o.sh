#!/bin/bash
# Pipelined staged table z-pass (zpipe): parity, then A/B on c3 / c2 / c5 table (RNG overlap on and off).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2o
mkdir -p $O
rm -f $O/ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "tuning or staging or golden" --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in c3 c2 c5; do
  timeout -k 10 300 python tools/ab.py --tune-a zpipe=0 --tune-b zpipe=1 --config $cfg --mode table --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a zpipe=0 --tune-b zpipe=1 --config c3 --mode table --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], d['A'], d['A_median_ms'], d['B'], d['B_median_ms'])"
