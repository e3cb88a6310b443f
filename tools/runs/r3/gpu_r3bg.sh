#!/bin/bash
# (zunroll 8 reverted since: profiles/r3/rejected/zunroll8; the key now clamps to 4) Table z-pass with a 16-tap body (zunroll 8: one wait per 16 taps' coefficients and noise): parity, A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bg
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "runtime_tuning or random_planes or fields_vs_oracle" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in c3 c2 native; do
  timeout -k 10 200 python3 tools/ab.py --config $cfg --mode table --rounds 9 --calls 20 --tune-a zunroll=4 --tune-b zunroll=8 \
    > $O/ab_$cfg.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$cfg.json'));print('$cfg', d['A'], d['A_median_ms']['zpass_ms'], d['A_median_ms']['wall_ms'], '|', d['B'], d['B_median_ms']['zpass_ms'], d['B_median_ms']['wall_ms'])"
done
DFAMD_RNG_OVERLAP=0 timeout -k 10 200 python3 tools/ab.py --config c3 --mode table --rounds 9 --calls 20 --tune-a zunroll=4 --tune-b zunroll=8 \
    > $O/ab_c3_alone.json || { echo "ab failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/ab_c3_alone.json'));print('c3 alone', d['A'], d['A_median_ms']['zpass_ms'], d['A_median_ms']['wall_ms'], '|', d['B'], d['B_median_ms']['zpass_ms'], d['B_median_ms']['wall_ms'])"
