#!/bin/bash
# Hand-off batching: the GPU suite (small planes now run epochs of 4 calls), then wall per call with
# hand-off batch 1 / 2 / 4 on the small planes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3i}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for cfg in "c1 packed" "c2 packed" "native packed" "c1 table" "c2 table" "native table"; do
  timeout -k 10 200 python3 tools/hb_ab.py $cfg 7 48 >> $O/hb_ab.jsonl 2>> $O/hb.err || { echo "failed $cfg"; tail -20 $O/hb.err; exit 1; }
  tail -1 $O/hb_ab.jsonl
done
