#!/bin/bash
# Kc with an all-needed fast loop: parity (dense forced on small planes, tuning matrix, whole c3 plane), then the
# c3 table serial kernel timeline (Kc was 20.4 us, profiles/r3/ad).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3aw
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_dense.py \
  -k "dense or runtime_tuning or random_planes or bitexact_vs_oracle" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullsize.py \
  -k "c3_whole" > $O/pytest_c3.log 2>&1 || { echo "pytest c3 failed"; tail -30 $O/pytest_c3.log; exit 1; }
tail -1 $O/pytest_c3.log
cd /tmp && export TMPDIR=/tmp
DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
   python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 20 > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/rocprof_split.py $O/prof/run_kernel_trace.csv | grep -E "rng|kernel,grid" 
rm -f $O/prof/run_kernel_trace.csv
