#!/bin/bash
# c2 packed (2048 row-pair tiles, ~3 waves per SIMD): 1 row per wave with the 8-deep load pipeline and/or the
# z-pass at a wave per component (zsplit), against the defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bi
mkdir -p $O
for b in "rows_per_wave=1,yunroll=8" "zsplit=1" "rows_per_wave=1,yunroll=8,zsplit=1" "rows_per_wave=1,yunroll=16"; do
  timeout -k 10 200 python3 tools/ab.py --config c2 --mode packed --rounds 11 --calls 20 --tune-a rows_per_wave=2,yunroll=2,zsplit=0 \
    --tune-b $b > $O/ab_$b.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$b.json'));a=d['A_median_ms'];b=d['B_median_ms'];print(d['A'], a['ypass_ms'], a['zpass_ms'], a['wall_ms'], '|', d['B'], b['ypass_ms'], b['zpass_ms'], b['wall_ms'])"
done
