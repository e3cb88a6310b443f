#!/bin/bash
# K3 batch skeleton on select-chain tables: parity, then standalone times (overlap off) with and without
# the transform (DFAMD_RNG_DEBUG 7), and in-process A/B against the sequential K3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r2k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export TMPDIR=/tmp
for f in 0 7; do
  (cd /tmp && DFAMD_RNG_OVERLAP=0 DFAMD_RNG_DEBUG=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv \
     -d $O/abl$f -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 20 > $O/abl$f.log 2>&1) || { echo "ablation $f failed"; tail -5 $O/abl$f.log; exit 1; }
  python3 - "$O/abl$f/run_kernel_stats.csv" $f <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if 'rng_generate' in x['Name'] or 'rng_count' in x['Name']:
        print('flags', sys.argv[2], '%-40s avg_us=%9.1f' % (x['Name'][:40], float(x['AverageNs']) / 1e3))
PY
done
cd "$GRAFT_REPO_ROOT"
for cfg in "c3 table" "c3 packed" "native table" "c1 table"; do
  set -- $cfg
  timeout -k 10 300 python tools/ab.py --tune-a gen_compact=0 --tune-b gen_compact=1 --config $1 --mode $2 --rounds 7 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], 'seq', d['A_median_ms'], 'compact', d['B_median_ms'])"
