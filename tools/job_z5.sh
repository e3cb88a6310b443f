set -o pipefail
# the original explicit z-pass tap steps restored: parity, VALU per call, c3 table alone
cd $GRAFT_REPO_ROOT
O=gpurun_out/z5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ghost.py tests/test_gpu_ahead.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/valu_issue.sh || exit 1
(cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 40 > $GRAFT_REPO_ROOT/$O/tr.log 2>&1) || exit 1
python3 tools/rocprof_split.py $O/tr/run_kernel_trace.csv > $O/tr.split.csv; grep "pass" $O/tr.split.csv | head -3
