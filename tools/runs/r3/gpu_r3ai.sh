#!/bin/bash
# The reference's grid in table mode (the drop-in default there): y-pass forms for its long chains (N_y <= 212).
# Default (2 rows per wave, group-ahead ydeep) against the 8-deep register ring (yunroll 8) at 1/2/4 rows per wave.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ai
mkdir -p $O
for b in "yunroll=8,rows_per_wave=1" "yunroll=8,rows_per_wave=2" "yunroll=8,rows_per_wave=4" "rows_per_wave=1" "rows_per_wave=4"; do
  for ov in 0 1; do
    DFAMD_RNG_OVERLAP=$ov timeout -k 10 200 python3 tools/ab.py --config native --mode table --rounds 9 --calls 20 \
      --tune-a yunroll=2,rows_per_wave=2 --tune-b $b > $O/ab_${b}_ov$ov.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_${b}_ov$ov.json'));print('ov$ov default', d['A_median_ms']['ypass_ms'], d['A_median_ms']['wall_ms'], '$b', d['B_median_ms']['ypass_ms'], d['B_median_ms']['wall_ms'])"
  done
done
