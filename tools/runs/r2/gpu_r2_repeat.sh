#!/bin/bash
# The GPU suite twice in a row on one box (flakiness check of the final code), then smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2rep}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_$i.log 2>&1 || { echo "pytest run $i failed"; grep -E "FAILED|Error" $O/pytest_$i.log | head; tail -3 $O/pytest_$i.log; exit 1; }
  tail -1 $O/pytest_$i.log
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
