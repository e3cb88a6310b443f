#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench command, per coefficient mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-prof}; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for mode in packed table; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/$mode -o run -- \
     python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline off --alt-modes off --coeff-mode $mode --steps 20 --warmup 3 "$@" \
     > $O/$mode.log 2>&1) || { echo "rocprof $mode failed"; tail -5 $O/$mode.log; exit 1; }
  grep '^{' $O/$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode bench-under-rocprof', d['value'], d['ms_per_step'])"
  python3 - "$O/$mode/run_kernel_stats.csv" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print('  %-32s calls=%5s avg_us=%9.1f' % (x['Name'][:32], x['Calls'], float(x['AverageNs']) / 1e3))
PY
done
