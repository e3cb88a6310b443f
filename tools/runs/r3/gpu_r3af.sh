#!/bin/bash
# Table y-pass rows per wave after the window path and register diet: 4 (default) vs 8 vs 2, same handle, c3/c5
# table, RNG overlap off (the y-pass alone) and on.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3af6
mkdir -p $O
for ov in 0 1; do
  for b in 6; do
    DFAMD_RNG_OVERLAP=$ov timeout -k 10 200 python3 tools/ab.py --config c3 --mode table --rounds 9 --calls 20 \
      --tune-a rows_per_wave=4 --tune-b rows_per_wave=$b > $O/ab_rpw${b}_ov$ov.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_rpw${b}_ov$ov.json'));print('overlap $ov rpw4', d['A_median_ms'], 'rpw$b', d['B_median_ms'])"
  done
done
