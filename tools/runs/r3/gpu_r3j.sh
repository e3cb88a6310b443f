#!/bin/bash
# K3a (dense generation) instruction breakdown: SQ_INSTS_VALU / SALU per dispatch under the timing-only
# ablations (DFAMD_RNG_DEBUG 1 no log/sqrt/div, 2 no stores, 4 no redraw, 7 all three), c3 table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3j}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for f in 0 1 2 4 7; do
  (cd /tmp && DFAMD_RNG_OVERLAP=0 DFAMD_RNG_DEBUG=$f timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES \
     --kernel-trace -d $O/f$f -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 4 > $O/f$f.log 2>&1) \
     || { echo "pmc $f failed"; tail -5 $O/f$f.log; exit 1; }
  python3 tools/pmc_summary.py $O/f$f rng_dense > $O/f$f.json
  python3 -c "
import json; d=json.load(open('$O/f$f.json'))
for k,v in d.items(): print('flags $f', k[:40], 'VALU %.2fM SALU %.2fM waves %d' % (v['SQ_INSTS_VALU']/1e6, v['SQ_INSTS_SALU']/1e6, v['SQ_WAVES']))"
done
