#!/bin/bash
# Compacted K3 skeleton: standalone times with timing-only ablations (DFAMD_RNG_DEBUG 7: no transform,
# no stores, no redraw; 8: append loop only; 15: both), c3 table, RNG overlap off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r2j
mkdir -p $O
export TMPDIR=/tmp
for f in 7 8 15; do
  (cd /tmp && DFAMD_RNG_OVERLAP=0 DFAMD_RNG_DEBUG=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv \
     -d $O/abl$f -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 20 > $O/abl$f.log 2>&1) || { echo "ablation $f failed"; tail -5 $O/abl$f.log; exit 1; }
  python3 - "$O/abl$f/run_kernel_stats.csv" $f <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if 'rng_' in x['Name']:
        print('flags', sys.argv[2], '%-40s avg_us=%9.1f' % (x['Name'][:40], float(x['AverageNs']) / 1e3))
PY
done
