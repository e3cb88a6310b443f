#!/bin/bash
# Kernel timelines of the small planes (c2, the reference's grid) in both modes: where a call's wall
# time goes between kernels (rocprofv3 kernel trace, both streams).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2ai}
mkdir -p $O
export TMPDIR=/tmp
for cm in "c2 packed" "c2 table" "native packed"; do
  set -- $cm
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$1_$2 -o run -- \
     python3 $GRAFT_REPO_ROOT/tools/plane_loop.py $1 $2 60 > $O/$1_$2.log 2>&1) || { echo "trace $cm failed"; tail -5 $O/$1_$2.log; exit 1; }
  python3 - $O/$1_$2/run_kernel_trace.csv "$cm" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
rows = [r for r in rows if 'dfamd' in r['Kernel_Name']][-200:]
t0 = int(rows[0]['Start_Timestamp'])
out = []
for r in rows[-40:]:
    s, e = int(r['Start_Timestamp']) - t0, int(r['End_Timestamp']) - t0
    out.append('%9.1f %9.1f %7.1f q%s %s' % (s / 1e3, e / 1e3, (e - s) / 1e3, r.get('Queue_Id', r.get('Stream_Id', '?')), r['Kernel_Name'][:60]))
print(sys.argv[2]); print('\n'.join(out))
PY
done
