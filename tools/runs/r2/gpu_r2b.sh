#!/bin/bash
# RNG rework check: GPU parity suite, then in-process A/B of the sequential vs compacted K3
# (K1's two-multiply screen is in both), and the standalone kernel times (overlap off) under rocprofv3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_writers.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "c3 table" "c3 packed" "native table" "native packed" "c1 table"; do
  set -- $cfg
  timeout -k 10 300 python tools/ab.py --tune-a gen_compact=0 --tune-b gen_compact=1 --config $1 --mode $2 --rounds 7 --calls 20 >> $O/ab_compact.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab_compact.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], 'seq', d['A_median_ms'], 'compact', d['B_median_ms'])"
export TMPDIR=/tmp
for gc in 0 1; do
  (cd /tmp && DFAMD_RNG_OVERLAP=0 DFAMD_GEN_COMPACT=$gc timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv \
     -d $GRAFT_REPO_ROOT/$O/prof_gc$gc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --coeff-mode table --cpu-baseline off \
     --alt-modes off --other-configs '' --parity off --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof_gc$gc.log 2>&1) \
     || { echo "rocprof failed"; tail -5 $O/prof_gc$gc.log; exit 1; }
  python3 - "$O/prof_gc$gc/run_kernel_stats.csv" $gc <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if 'rng' in x['Name'] or 'pass' in x['Name']:
        print('gc', sys.argv[2], '%-40s calls=%5s avg_us=%9.1f' % (x['Name'][:40], x['Calls'], float(x['AverageNs']) / 1e3))
PY
done
