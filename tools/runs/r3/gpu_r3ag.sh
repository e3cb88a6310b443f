#!/bin/bash
# K3a fast chunks (host-built destinations for chunks inside one r_ys array): parity (forced dense on small planes,
# tuning matrix, whole c3 plane vs the oracle), then same-handle A/B k3a_fast 0 vs 1 on c3/c5 table, overlap off/on.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ag
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "dense_fast or runtime_tuning or bitexact_vs_oracle or native" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullsize.py \
  -k "c3" > $O/pytest_c3.log 2>&1 || { echo "pytest c3 failed"; tail -30 $O/pytest_c3.log; exit 1; }
tail -1 $O/pytest_c3.log
for ov in 0 1; do
  for cfg in c3 c5; do
    DFAMD_RNG_OVERLAP=$ov timeout -k 10 200 python3 tools/ab.py --config $cfg --mode table --rounds 9 --calls 20 \
      --tune-a k3a_fast=0 --tune-b k3a_fast=1 > $O/ab_${cfg}_ov$ov.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_${cfg}_ov$ov.json'));print('$cfg overlap $ov fast0', d['A_median_ms'], 'fast1', d['B_median_ms'])"
  done
done
