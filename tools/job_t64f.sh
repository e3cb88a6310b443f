set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/t64f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ghost.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "native_grid_bitexact or runtime_tuning or ghost_strips" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 5 100 ./tools/fp64_lat > $O/fp64_lat.jsonl; cat $O/fp64_lat.jsonl
for v in "ylds=2 rows_per_wave=1" "ylds=3 yt_rows=1 yt_pd=2" "ylds=3 yt_rows=1 yt_pd=4" "ylds=3 yt_rows=2 yt_chunk=16 yt_pd=2" "ylds=3 yt_rows=2 yt_chunk=8 yt_pd=2" "ylds=3 yt_rows=2 yt_chunk=8 yt_pd=4" "ylds=3 yt_rows=4 yt_pd=2"; do
  n=$(echo $v | tr ' =' '_-')
  (cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native table 200 $v > $GRAFT_REPO_ROOT/$O/tr_$n.log 2>&1) || exit 1
  python3 tools/rocprof_split.py $O/tr_$n/run_kernel_trace.csv > $O/tr_$n.split.csv; echo "== $v"; grep "ypass" $O/tr_$n.split.csv | head -1
done
