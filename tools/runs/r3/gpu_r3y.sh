#!/bin/bash
# Table y-pass: the deep (a group ahead) pipeline with one shared coefficient window per group on uniform-N
# tiles (ywindow 1, new) vs per-row coefficient loads (ywindow 0); parity first; same-handle A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3y
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "runtime_tuning or native or bitexact_vs_oracle or table" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cm in "c3 table" "c2 table" "native table" "c1 table"; do
  set -- $cm
  timeout -k 10 200 python3 tools/ab.py --config $1 --mode $2 --rounds 9 --calls 20 --tune-a ywindow=0 --tune-b ywindow=1 \
    > $O/ab_$1_$2.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2.json'));print('$1 $2 ywindow0', d['A_median_ms'], 'ywindow1', d['B_median_ms'])"
  DFAMD_RNG_OVERLAP=0 timeout -k 10 200 python3 tools/ab.py --config $1 --mode $2 --rounds 9 --calls 20 --tune-a ywindow=0 --tune-b ywindow=1 \
    > $O/ab_$1_$2_serial.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2_serial.json'));print('   overlap off ywindow0', d['A_median_ms'], 'ywindow1', d['B_median_ms'])"
done
