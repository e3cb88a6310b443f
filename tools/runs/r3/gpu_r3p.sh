#!/bin/bash
# Row-pair y-pass dispatch order on the reference's grid (packed): ascending rows (ycoop_order 0) against
# heaviest-group-first orders (groups of 1, 4, 16 tiles), same handle (tools/ab.py --tune-*), plus parity.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3p
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "native or runtime_tuning" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for g in 1 4 16 64; do
  timeout -k 10 120 python3 tools/ab.py --config native --mode packed --rounds 11 --calls 20 \
    --tune-a ycoop_order=0 --tune-b ycoop_order=$g > $O/ab_order_$g.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_order_$g.json'));print('order $g', d['A_median_ms'], d['B_median_ms'])"
done
