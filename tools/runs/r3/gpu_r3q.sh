#!/bin/bash
# Timing-only ablations of the row-pair y-pass on the reference's grid (packed): noise loads, coefficient
# loads, both, or the LDS tap-order sum replaced; ycoop_order 4 (heaviest groups first) on every library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3q
mkdir -p $O
L=$GRAFT_REPO_ROOT/digital-filtering_amd
for i in 1 2; do
  for v in "" _nonoise _nocoef _nocoefnoise _nosum; do
    DFAMD_LIB=$L/libdfamd$v.so timeout -k 10 120 python3 tools/ab.py --config native --mode packed --rounds 9 --calls 20 \
      --tune-a ycoop_order=4 --tune-b ycoop_order=4,ycoop=8 > $O/ab${v}_$i.json || { echo "ab $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab${v}_$i.json'));print('lib$v', d['A_median_ms']['ypass_ms'], d['A_median_ms']['wall_ms'], 'ycoop8', d['B_median_ms']['ypass_ms'])"
  done
done
