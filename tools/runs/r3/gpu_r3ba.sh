#!/bin/bash
# ypre 2 (reverted since: profiles/r3/rejected/ypre2; the key now clamps to 1): the next call's y-pass on its own stream (started by its generation's event), so consecutive
# calls' y-passes run back to back beside the z-passes. Parity, then same-handle A/B ypre 0 vs 2 on the
# reference's grid and c3/c2 packed (and native table for the record).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ba
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "ypass_prefetch or runtime_tuning or handoff" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cm in "native packed" "c2 packed" "c3 packed" "native table"; do
  set -- $cm
  timeout -k 10 200 python3 tools/ab.py --config $1 --mode $2 --rounds 9 --calls 20 --tune-a ypre=0 --tune-b ypre=2 \
    > $O/ab_$1_$2.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2.json'));print('$1 $2 ypre0', d['A_median_ms'], 'ypre2', d['B_median_ms'])"
done
