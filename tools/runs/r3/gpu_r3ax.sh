#!/bin/bash
# Hand-off batch drop to 1 after a loaded stream state (and the return 16 calls later): the hand-off, drop-in
# (two C++ objects on one stream), checkpoint/resume and tuning tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ax
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  tests/test_gpu_dropin.py tests/test_fortran.py -m gpu -k "handoff or cpp or checkpoint or resume or runtime_tuning or rng_state or ypass_prefetch or fortran" \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
