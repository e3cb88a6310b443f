set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/t64e; mkdir -p $O
for v in "ylds=3 yt_rows=1 yt_pd=2" "ylds=3 yt_rows=1 yt_pd=4" "ylds=3 yt_rows=2 yt_chunk=16 yt_pd=2" "ylds=3 yt_rows=2 yt_chunk=16 yt_pd=4" "ylds=3 yt_rows=2 yt_chunk=8 yt_pd=2" "ylds=3 yt_rows=2 yt_chunk=8 yt_pd=4"; do
  n=$(echo $v | tr ' =' '_-')
  (cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native table 200 $v > $GRAFT_REPO_ROOT/$O/tr_$n.log 2>&1) || exit 1
  python3 tools/rocprof_split.py $O/tr_$n/run_kernel_trace.csv > $O/tr_$n.split.csv; echo "== $v"; grep "ypass\|zpass\|rng_" $O/tr_$n.split.csv | head -5
done
for v in "gen_dense=2 fuse_plan=0 gen_split=1" "gen_split=8" "gen_split=16"; do
  n=$(echo $v | tr ' =' '_-')
  (cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/rg_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native table 200 $v > $GRAFT_REPO_ROOT/$O/rg_$n.log 2>&1) || exit 1
  python3 tools/rocprof_split.py $O/rg_$n/run_kernel_trace.csv > $O/rg_$n.split.csv; echo "== $v"; grep "rng_" $O/rg_$n.split.csv | head -5
done
