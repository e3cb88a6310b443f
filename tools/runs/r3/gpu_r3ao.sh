#!/bin/bash
# The reference's grid in table mode: 2 rows per wave (default so far) vs 1 row per wave with the deep noise
# ring (ydepth 1), same handle, overlap on (the real call), 3 repeats of 11 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ao
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python3 tools/ab.py --config native --mode table --rounds 11 --calls 30 \
    --tune-a rows_per_wave=2,ydepth=1 --tune-b rows_per_wave=1,ydepth=1 > $O/ab_$i.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$i.json'));print('rpw2', d['A_median_ms']['wall_ms'], d['A_min_ms']['wall_ms'], 'rpw1', d['B_median_ms']['wall_ms'], d['B_min_ms']['wall_ms'])"
done
