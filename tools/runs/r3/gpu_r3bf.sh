#!/bin/bash
# LDS-staged table y-pass at 4 rows per wave with one coefficient window for the wave's rows (uniform N):
# parity, then c3 / c2 A/B against the per-wave form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bf
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "native_grid_bitexact or runtime_tuning or random_planes" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cm in "c3 4" "c3 8" "c2 4"; do
  set -- $cm
  timeout -k 10 200 python3 tools/ab.py --config $1 --mode table --rounds 9 --calls 20 --tune-a ylds=0,rows_per_wave=4 \
    --tune-b ylds=1,rows_per_wave=$2 > $O/ab_$1_r$2.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_r$2.json'));print('$1', d['A'], d['A_median_ms']['ypass_ms'], d['A_median_ms']['wall_ms'], '|', d['B'], d['B_median_ms']['ypass_ms'], d['B_median_ms']['wall_ms'])"
done
