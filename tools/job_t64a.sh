set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/t64a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dense.py tests/test_gpu_rungen.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/ab_multi.py --config native --mode table --tune ylds=2,rows_per_wave=1 --tune ylds=3,yt_rows=1 --tune ylds=3,yt_rows=2 --tune ylds=3,yt_rows=4 --tune ylds=3,yt_rows=8 > $O/ab.log 2>&1; rc=$?; cat $O/ab.log | grep tune; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 380 --timeout-method thread -k "vs_reference" > $O/tests_c3ref.log 2>&1; rc=$?; tail -3 $O/tests_c3ref.log; exit $rc
