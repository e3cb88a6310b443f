#!/bin/bash
# Table y-pass with LDS-staged noise (ylds): parity, then same-handle A/B ylds 0 vs 1 (rows per wave 1/2/4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bc
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "native_grid_bitexact or runtime_tuning or random_planes or golden" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cm in "c3 4" "c3 2" "native 1" "native 2" "c2 4" "c2 2"; do
  set -- $cm
  timeout -k 10 200 python3 tools/ab.py --config $1 --mode table --rounds 9 --calls 20 --tune-a ylds=0 --tune-b ylds=1,rows_per_wave=$2 \
    > $O/ab_$1_r$2.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_r$2.json'));print('$1', d['A'], d['A_median_ms'], '|', d['B'], d['B_median_ms'])"
done
