#!/bin/bash
# Table y-pass at 4 rows per wave with the noise ring 2 groups (8 rows) ahead (ydepth 1) vs 1 group (0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bk
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "runtime_tuning or random_planes or fields_vs_oracle or native_grid_bitexact" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in c3 c2; do
  timeout -k 10 200 python3 tools/ab.py --config $cfg --mode table --rounds 11 --calls 20 --tune-a ydepth=0 --tune-b ydepth=1 \
    > $O/ab_$cfg.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$cfg.json'));a=d['A_median_ms'];b=d['B_median_ms'];print('$cfg', d['A'], a['ypass_ms'], a['wall_ms'], '|', d['B'], b['ypass_ms'], b['wall_ms'])"
done
DFAMD_RNG_OVERLAP=0 timeout -k 10 200 python3 tools/ab.py --config c3 --mode table --rounds 11 --calls 20 --tune-a ydepth=0 --tune-b ydepth=1 \
    > $O/ab_c3_alone.json || { echo "ab failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/ab_c3_alone.json'));a=d['A_median_ms'];b=d['B_median_ms'];print('c3 alone', d['A'], a['ypass_ms'], a['wall_ms'], '|', d['B'], b['ypass_ms'], b['wall_ms'])"
