#!/bin/bash
# z-pass register budget (zocc 8: 8 waves per SIMD, 54/64 VGPRs) against the default (76 VGPRs, 6 waves), same
# handle, interleaved rounds: c3 packed (the headline K5), c2 packed, c3/c2 table. Parity subset first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ac
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "runtime_tuning or bitexact_vs_oracle" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cm in "c3 packed" "c3 packed" "c2 packed" "c3 table" "c2 table" "native packed"; do
  set -- $cm
  timeout -k 10 200 python3 tools/ab.py --config $1 --mode $2 --rounds 9 --calls 10 --tune-a zocc=0 --tune-b zocc=8 \
    > $O/ab_$1_$2.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2.json'));print('$1 $2 zocc0', d['A_median_ms'], 'zocc8', d['B_median_ms'])"
done
