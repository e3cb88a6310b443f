#!/bin/bash
# glibc's own log in K3 (fast_log 2): bit-exact normals and fields against the oracle and the
# reference's fixtures, then the cost against log_r2 (fast_log 1) on the table-mode planes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2ah}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "bitexact or noise_arrays or golden or rng_stream" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cm in "c3 table" "native table" "c2 table" "c3 packed"; do
  set -- $cm
  timeout -k 10 300 python tools/ab.py --tune-a fast_log=1 --tune-b fast_log=2 --config $1 --mode $2 --rounds 9 --calls 30 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a fast_log=1 --tune-b fast_log=2 --config c3 --mode table --rounds 9 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
  || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); a=d['A_median_ms']; b=d['B_median_ms']; print(d['config'], d['mode'], d['A'], a.get('rng_ms'), a['wall_ms'], '|', d['B'], b.get('rng_ms'), b['wall_ms'])"
