#!/bin/bash
# The full-size suite, with the new whole-plane c3 oracle comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3l}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=0 > $O/pytest_fullsize.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_fullsize.log; exit 1; }
grep -E "PASS|FAIL|passed|failed|s call" $O/pytest_fullsize.log | tail -20
