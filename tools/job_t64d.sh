set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/t64d; mkdir -p $O
for v in "ylds=2 rows_per_wave=1 nt_stores=0" "ylds=3 yt_rows=1 yt_pd=2 nt_stores=0" "ylds=3 yt_rows=2 yt_chunk=16 yt_pd=2 nt_stores=0" "ylds=3 yt_rows=2 yt_chunk=8 yt_pd=2 nt_stores=0" "ylds=3 yt_rows=4 yt_pd=2 nt_stores=0"; do
  n=$(echo $v | tr ' =' '_-')
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native table 200 $v > $GRAFT_REPO_ROOT/$O/tr_$n.log 2>&1) || exit 1
  python3 tools/rocprof_split.py $O/tr_$n/run_kernel_trace.csv > $O/tr_$n.split.csv; echo "== $v"; grep "ypass\|zpass\|rng_" $O/tr_$n.split.csv | head -5
done
timeout -k 10 300 python3 tools/ab_multi.py --config native --mode table --tune ylds=2,rows_per_wave=1,nt_stores=1 --tune ylds=2,rows_per_wave=1,nt_stores=0 --tune ylds=3,yt_rows=1,nt_stores=0 --tune ylds=3,yt_rows=2,yt_chunk=16,nt_stores=0 > $O/ab.log 2>&1; rc=$?; cat $O/ab.log | grep tune; exit $rc
