#!/bin/bash
# What bounds the table y-pass on the reference's grid (long chains)? Timing-only ablations: table coefficients
# as a constant (no scalar loads, DF_ABLATE_TCOEF) and noise from registers (DF_ABLATE_NOISE); rows per wave 2, 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3an
mkdir -p $O
L=$GRAFT_REPO_ROOT/digital-filtering_amd
for v in "" _tcoef _tnoise; do
  DFAMD_LIB=$L/libdfamd$v.so DFAMD_RNG_OVERLAP=0 timeout -k 10 200 python3 tools/ab.py --config native --mode table --rounds 7 --calls 20 \
    --tune-a rows_per_wave=2 --tune-b rows_per_wave=1 > $O/ab$v.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab$v.json'));print('lib$v rpw2', d['A_median_ms']['ypass_ms'], 'rpw1', d['B_median_ms']['ypass_ms'])"
  DFAMD_LIB=$L/libdfamd$v.so DFAMD_RNG_OVERLAP=0 timeout -k 10 200 python3 tools/ab.py --config c3 --mode table --rounds 5 --calls 10 \
    > $O/ab_c3$v.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_c3$v.json'));print('   c3 lib$v', d['A_median_ms']['ypass_ms'], d['A_median_ms']['zpass_ms'])"
done
