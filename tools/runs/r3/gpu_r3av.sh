#!/bin/bash
# The reference's grid now batches its hand-offs (hb 4): GPU tests that drive it (golden/oracle, drop-in C++,
# Fortran, writers, statistics, hand-off epochs), then the default handle's wall per call (hb_ab).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3av
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  tests/test_gpu_dropin.py tests/test_fortran.py tests/test_writers.py -m gpu -k "native or dropin or cpp or fortran or writer or rms or handoff or golden" \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/hb_ab.py native packed 9 48 > $O/hb_native_packed.json && cat $O/hb_native_packed.json
timeout -k 10 300 python3 tools/hb_ab.py native table 9 48 > $O/hb_native_table.json && cat $O/hb_native_table.json
