#!/bin/bash
# LDS-staged table y-pass with 1-3 noise chunks in flight (ylds 1/2/3): parity, then same-handle A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bd
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "native_grid_bitexact or runtime_tuning or random_planes" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cm in "native 1 1 1" "native 1 2 1" "native 1 3 1" "native 2 3 1" "c3 4 2 4" "c3 4 3 4" "c3 2 3 4" "c2 4 3 4" "c2 1 3 4"; do
  set -- $cm
  timeout -k 10 200 python3 tools/ab.py --config $1 --mode table --rounds 9 --calls 20 --tune-a ylds=0,rows_per_wave=$4 \
    --tune-b ylds=$3,rows_per_wave=$2 > $O/ab_$1_r$2_l$3.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_r$2_l$3.json'));print('$1', d['A'], d['A_median_ms']['ypass_ms'], d['A_median_ms']['wall_ms'], '|', d['B'], d['B_median_ms']['ypass_ms'], d['B_median_ms']['wall_ms'])"
done
