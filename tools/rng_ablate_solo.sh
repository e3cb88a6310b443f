#!/bin/bash
# RNG generate ablation for one z-strip rank of an N-way split (timing only; flags != 0 give wrong
# results): 1 no log/sqrt/div, 2 no stores, 4 no draw recompute. Usage: tools/rng_ablate_solo.sh N
set -o pipefail
N=${1:-8}
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/rng_ablate_solo_n$N; mkdir -p $O
for f in 0 7; do
  (cd /tmp && DFAMD_RNG_OVERLAP=0 DFAMD_RNG_DEBUG=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $O/f$f -o run -- python3 $GRAFT_REPO_ROOT/tools/solo_rank.py $N 0 table 10 > $O/f$f.log 2>&1) || { echo fail $f; tail -3 $O/f$f.log; exit 1; }
  python3 - "$O/f$f/run_kernel_stats.csv" $f <<'PY'
import csv, sys
d = {x['Name'].split('(')[0].replace('dfamd::', ''): float(x['AverageNs']) / 1e3 for x in csv.DictReader(open(sys.argv[1]))}
print('flags', sys.argv[2], 'generate_us %.1f count_us %.1f' % (d.get('rng_generate_kernel', -1), d.get('rng_count_kernel', -1)))
PY
done
