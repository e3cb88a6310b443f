#!/bin/bash
# Table-driven log in K3: parity suite, standalone RNG kernel times, in-process A/B on c3 table/packed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r2p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
grep "max ulp" $O/pytest.log || true
export TMPDIR=/tmp
for fl in 0 1; do
  (cd /tmp && DFAMD_RNG_OVERLAP=0 DFAMD_FAST_LOG=$fl timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $O/prof$fl -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 20 > $O/prof$fl.log 2>&1) || { echo "prof $fl failed"; tail -5 $O/prof$fl.log; exit 1; }
  python3 - "$O/prof$fl/run_kernel_stats.csv" $fl <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    n = x['Name']
    if 'rng_generate' in n or 'rng_count' in n or 'pass_kernel' in n:
        print('fast_log', sys.argv[2], '%-60s avg_us=%9.1f' % (n[:60], float(x['AverageNs']) / 1e3))
PY
  rm -f $O/prof$fl/run_kernel_trace.csv
done
cd "$GRAFT_REPO_ROOT"
for cfg in "c3 table" "c3 packed" "native table"; do
  set -- $cfg
  timeout -k 10 300 python tools/ab.py --tune-a fast_log=0 --tune-b fast_log=1 --config $1 --mode $2 --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], d['A'], d['A_median_ms'], d['B'], d['B_median_ms'])"
