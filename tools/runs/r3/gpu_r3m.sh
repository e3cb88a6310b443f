#!/bin/bash
# Hand-off batching: generations spread one per step (hb ahead) against one burst per epoch; parity suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3m}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dense.py tests/test_gpu_dropin.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "c1 packed" "c2 packed" "native packed" "c1 table" "c2 table" "native table"; do
  timeout -k 10 200 python3 tools/hb_ab.py $cfg 7 48 >> $O/hb_ab.jsonl 2>> $O/hb.err || { echo "failed $cfg"; tail -20 $O/hb.err; exit 1; }
  tail -1 $O/hb_ab.jsonl
done
