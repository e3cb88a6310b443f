set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/t64b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ghost.py tests/test_gpu_dense.py tests/test_gpu_rungen.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "native or runtime_tuning or ghost or dense or rungen" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/ab_multi.py --config native --mode table --tune ylds=2,rows_per_wave=1 --tune ylds=3,yt_rows=1 --tune ylds=3,yt_rows=2,yt_chunk=8 --tune ylds=3,yt_rows=2,yt_chunk=16 --tune ylds=3,yt_rows=4 > $O/ab.log 2>&1; rc=$?; cat $O/ab.log | grep tune; [ $rc -ne 0 ] && exit $rc
for v in "ylds=3 yt_rows=1" "ylds=3 yt_rows=2 yt_chunk=8" "ylds=3 yt_rows=2 yt_chunk=16" "ylds=3 yt_rows=4"; do
  n=$(echo $v | tr ' =' '_-')
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native table 200 $v > $GRAFT_REPO_ROOT/$O/tr_$n.log 2>&1) || exit 1
  python3 tools/rocprof_split.py $O/tr_$n/run_kernel_trace.csv > $O/tr_$n.split.csv; echo "== $v"; grep ypass_t64 $O/tr_$n.split.csv
done
