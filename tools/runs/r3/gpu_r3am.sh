#!/bin/bash
# Table y-pass at 1-2 rows per wave with the noise 4 groups ahead (ydepth 1) vs the group-ahead pipeline
# (ydepth 0): parity (tuning matrix, whole reference grid vs the oracle), then same-handle A/B on the
# reference's grid in table mode (the drop-in default there) at 2 and 1 rows per wave.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3am
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "runtime_tuning or native or random_planes" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for ov in 1 0; do
  for rpw in 2 1; do
    DFAMD_RNG_OVERLAP=$ov timeout -k 10 200 python3 tools/ab.py --config native --mode table --rounds 9 --calls 20 \
      --tune-a ydepth=0,rows_per_wave=$rpw --tune-b ydepth=1,rows_per_wave=$rpw > $O/ab_rpw${rpw}_ov$ov.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_rpw${rpw}_ov$ov.json'));print('ov$ov rpw$rpw depth0', d['A_median_ms'], 'depth1', d['B_median_ms'])"
  done
done
