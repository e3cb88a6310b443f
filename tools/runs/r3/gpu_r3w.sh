#!/bin/bash
# Reference's grid, packed: the row-pair block form (ycoop 7, default) against per-wave y-passes with deeper
# register rings (yunroll 16/32, 1 or 2 rows per wave); RNG overlap off so the y-pass is timed alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3w
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "runtime_tuning" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for b in "ycoop=0,rows_per_wave=1,yunroll=8" "ycoop=0,rows_per_wave=1,yunroll=16" "ycoop=0,rows_per_wave=1,yunroll=32" \
         "ycoop=0,rows_per_wave=2,yunroll=8" "ycoop=0,rows_per_wave=2,yunroll=16" "ycoop=0,rows_per_wave=2,yunroll=32" \
         "ycoop=0,rows_per_wave=2,yunroll=16,heavy_first=0" "ycoop=0,rows_per_wave=1,yunroll=32,heavy_first=0"; do
  DFAMD_RNG_OVERLAP=0 timeout -k 10 120 python3 tools/ab.py --config native --mode packed --rounds 7 --calls 20 \
    --tune-a ycoop=7 --tune-b $b > $O/ab_$b.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$b.json'));print('ycoop7', d['A_median_ms']['ypass_ms'], '$b', d['B_median_ms']['ypass_ms'])"
done
