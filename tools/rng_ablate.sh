#!/bin/bash
# Timing-only ablation of the RNG generate kernel (results are wrong with flags != 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/rng_ablate; mkdir -p $O
for f in 0 1 2 4 7; do
  (cd /tmp && DFAMD_RNG_OVERLAP=0 DFAMD_RNG_DEBUG=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv \
     -d $O/f$f -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline off --coeff-mode table --alt-modes off --steps 10 --warmup 2 > $O/f$f.log 2>&1) || { echo fail $f; tail -3 $O/f$f.log; exit 1; }
  python3 - "$O/f$f/run_kernel_stats.csv" $f <<'PY'
import csv, sys
d = {x['Name']: float(x['AverageNs']) / 1e3 for x in csv.DictReader(open(sys.argv[1]))}
print('flags', sys.argv[2], 'generate_us %.1f count_us %.1f' % (d.get('rng_generate_kernel', -1), d.get('rng_count_kernel', -1)))
PY
done
