#!/bin/bash
# LDS-staged table y-pass on the reference's grid: 4 waves x 16-row chunks (default) vs 8 waves (8 rows per
# block) with 16- or 32-row chunks. Parity first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3be
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "native_grid_bitexact or runtime_tuning or random_planes" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for b in "ylds_nw=8,ylds_ch=16" "ylds_nw=8,ylds_ch=32" "ylds=3" "ylds=1"; do
  timeout -k 10 200 python3 tools/ab.py --config native --mode table --rounds 11 --calls 20 --tune-a ylds=2,ylds_nw=4,ylds_ch=16 \
    --tune-b ylds=2,$b > $O/ab_$b.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$b.json'));print(d['A'], d['A_median_ms']['ypass_ms'], d['A_median_ms']['wall_ms'], '|', d['B'], d['B_median_ms']['ypass_ms'], d['B_median_ms']['wall_ms'])"
done
