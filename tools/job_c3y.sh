set -o pipefail
# c3 table: the y-pass forms isolated (RNG on the sweep stream) and the call A/B of the default against ylds 3
cd $GRAFT_REPO_ROOT
O=gpurun_out/c3y; mkdir -p $O
for v in "ylds=0" "ylds=3 yt_rows=1" "ylds=3 yt_rows=2 yt_chunk=16" "ylds=3 yt_rows=2 yt_chunk=8" "ylds=2 rows_per_wave=1"; do
  n=$(echo $v | tr ' =' '_-')
  (cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 60 $v > $GRAFT_REPO_ROOT/$O/tr_$n.log 2>&1) || exit 1
  python3 tools/rocprof_split.py $O/tr_$n/run_kernel_trace.csv > $O/tr_$n.split.csv; echo "== $v"; grep "ypass\|zpass\|rng_" $O/tr_$n.split.csv | head -5
done
timeout -k 10 300 python3 tools/ab.py --config c3 --mode table --tune-a ylds=0 --tune-b ylds=3,yt_rows=2,yt_chunk=16 --events 0 > $O/ab1.json 2>&1; cat $O/ab1.json | tail -3
