#!/bin/bash
# Per-call stream hand-off events with a device-scope release (DFAMD_EVENT_SCOPE=device) or no system
# fence (nofence) against the default: parity with the setting on, then A/B on small and large planes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2aj}
mkdir -p $O
for sc in device nofence; do
  DFAMD_EVENT_SCOPE=$sc timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "bitexact or golden or rng_stream or zstage" > $O/pytest_$sc.log 2>&1 || { echo "pytest $sc failed"; tail -30 $O/pytest_$sc.log; exit 1; }
  tail -1 $O/pytest_$sc.log
done
for cm in "c2 packed" "native packed" "c2 table" "native table" "c3 table" "c3 packed"; do
  set -- $cm
  timeout -k 10 300 python tools/ab.py --a DFAMD_EVENT_SCOPE=system --b DFAMD_EVENT_SCOPE=device --config $1 --mode $2 --rounds 9 --calls 40 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
  timeout -k 10 300 python tools/ab.py --a DFAMD_EVENT_SCOPE=system --b DFAMD_EVENT_SCOPE=nofence --config $1 --mode $2 --rounds 9 --calls 40 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); a=d['A_median_ms']; b=d['B_median_ms']; print(d['config'], d['mode'], d['A'], a['wall_ms'], '|', d['B'], b['wall_ms'])"
