#!/bin/bash
# Row-pair y-pass (ycoop 7) on short-chain packed planes, whole call with the RNG overlapped: c3 (x3), c5, c2;
# same handle; ycoop_order 0 and 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3aq
mkdir -p $O
for cfg in c3 c3 c3 c5 c2; do
  for ord in 0 4; do
    timeout -k 10 300 python3 tools/ab.py --config $cfg --mode packed --rounds 7 --calls 10 \
      --tune-a ycoop=0 --tune-b ycoop=7,ycoop_order=$ord > $O/ab_${cfg}_o$ord.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_${cfg}_o$ord.json'));print('$cfg ycoop0', d['A_median_ms']['ypass_ms'], d['A_median_ms']['wall_ms'], 'ycoop7 order$ord', d['B_median_ms']['ypass_ms'], d['B_median_ms']['wall_ms'])"
  done
done
