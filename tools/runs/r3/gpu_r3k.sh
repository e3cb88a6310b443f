#!/bin/bash
# K3a with per-chunk destinations: parity (dense + parity suites), instruction counts (flags 0 and 7),
# c3 table A/B against the compacted K3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3k}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export TMPDIR=/tmp
for f in 0 7; do
  (cd /tmp && DFAMD_RNG_OVERLAP=0 DFAMD_RNG_DEBUG=$f timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES \
     --kernel-trace -d $O/f$f -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 4 > $O/f$f.log 2>&1) \
     || { echo "pmc $f failed"; tail -5 $O/f$f.log; exit 1; }
  python3 tools/pmc_summary.py $O/f$f rng_dense > $O/f$f.json
  python3 -c "
import json; d=json.load(open('$O/f$f.json'))
for k,v in d.items(): print('flags $f', k[:40], 'VALU %.2fM SALU %.2fM waves %d' % (v['SQ_INSTS_VALU']/1e6, v['SQ_INSTS_SALU']/1e6, v['SQ_WAVES']))"
done
timeout -k 10 300 python3 tools/ab.py --torch --config c3 --mode table --rounds 9 --tune-a gen_dense=0 --tune-b gen_dense=1 \
  > $O/ab_dense.json 2> $O/ab.err || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ab_dense.json')); print('A compact', d['A_median_ms'], 'B dense', d['B_median_ms'])"
