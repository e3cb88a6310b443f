#!/bin/bash
# Is the row-pair block y-pass's access pattern itself slower than the per-wave form? c3 packed (short chains,
# 16k tiles) with ycoop 0 (per-wave, default there) vs 7 (row pairs), same handle, RNG overlap off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ap
mkdir -p $O
DFAMD_RNG_OVERLAP=0 timeout -k 10 200 python3 tools/ab.py --config c3 --mode packed --rounds 7 --calls 10 \
  --tune-a ycoop=0 --tune-b ycoop=7 > $O/ab_c3.json || { echo "ab failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/ab_c3.json'));print('c3 ycoop0', d['A_median_ms']['ypass_ms'], 'ycoop7', d['B_median_ms']['ypass_ms'])"
DFAMD_RNG_OVERLAP=0 timeout -k 10 200 python3 tools/ab.py --config c3 --mode packed --rounds 7 --calls 10 \
  --tune-a ycoop=0 --tune-b ycoop=7,ycoop_map=1 > $O/ab_c3_map1.json || { echo "ab failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/ab_c3_map1.json'));print('c3 ycoop0', d['A_median_ms']['ypass_ms'], 'ycoop7 map1', d['B_median_ms']['ypass_ms'])"
