#!/bin/bash
# Dense noise generation: parity (new dense tests + the parity suite), then c3 table A/B of the
# compacted K3 (gen_dense 0) against the dense form (1), overlapped and standalone, and a rocprofv3
# kernel-stats pass of the standalone A/B (per-kernel times of Kc / K3a / K3b).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3b}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/ab.py --torch --config c3 --mode table --rounds 9 --tune-a gen_dense=0 --tune-b gen_dense=1 \
  > $O/ab_dense_c3_table.json 2> $O/ab.err || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
cat $O/ab_dense_c3_table.json
DFAMD_RNG_OVERLAP=0 timeout -k 10 300 python3 tools/ab.py --torch --config c3 --mode table --rounds 9 --tune-a gen_dense=0 \
  --tune-b gen_dense=1 > $O/ab_dense_c3_table_serial.json 2> $O/ab2.err || { echo "ab2 failed"; tail -20 $O/ab2.err; exit 1; }
cat $O/ab_dense_c3_table_serial.json
timeout -k 10 300 python3 tools/ab.py --torch --config c3 --mode packed --rounds 7 --tune-a gen_dense=0 --tune-b gen_dense=1 \
  > $O/ab_dense_c3_packed.json 2> $O/ab3.err || { echo "ab3 failed"; tail -20 $O/ab3.err; exit 1; }
cat $O/ab_dense_c3_packed.json
export TMPDIR=/tmp
for d in 0 1; do
(cd /tmp && DFAMD_RNG_OVERLAP=0 DFAMD_GEN_DENSE=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
   -d $O/prof_d$d -o run -- python3 $GRAFT_REPO_ROOT/tools/ab.py --config c3 --mode table --rounds 3 > $O/prof_d$d.log 2>&1) \
   || { echo "rocprof $d failed"; tail -5 $O/prof_d$d.log; exit 1; }
python3 - $O/prof_d$d/run_kernel_stats.csv $d <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print('dense', sys.argv[2], x['Name'].split('(')[0].replace('dfamd::', '')[:40].ljust(40), 'avg_us %.1f' % (float(x['AverageNs']) / 1e3), 'calls', x['Calls'])
PY
rm -f $O/prof_d$d/run_kernel_trace.csv
done
