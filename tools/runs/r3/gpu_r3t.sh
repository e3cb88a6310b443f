#!/bin/bash
# Which XCD's run sets the row-pair y-pass time on the reference's grid? Timing-only variants that run one
# XCD's tiles alone (only0/3/7) or all but XCD 7's (skip7); RNG overlap off; the run boundaries printed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3t
mkdir -p $O
L=$GRAFT_REPO_ROOT/digital-filtering_amd
for v in "" _only0 _only3 _only7 _skip7; do
  DFAMD_LIB=$L/libdfamd$v.so DFAMD_RNG_OVERLAP=0 timeout -k 10 120 python3 tools/ab.py --config native --mode packed --rounds 7 --calls 20 \
    --tune-a ycoop_ovh=0 --tune-b ycoop_ovh=128 > $O/ab$v.json || { echo "ab $v failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab$v.json'));print('lib$v ovh0', d['A_median_ms']['ypass_ms'], 'ovh128', d['B_median_ms']['ypass_ms'])"
done
