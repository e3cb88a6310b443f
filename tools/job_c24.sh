set -o pipefail
# ypass_t64 with 24-row chunks: parity, kernel alone, call A/B (60-call windows, both orders)
cd $GRAFT_REPO_ROOT
O=gpurun_out/c24; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "native_grid or runtime_tuning" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for v in "yt_chunk=16" "yt_chunk=24"; do
  n=$(echo $v | tr ' =' '_-')
  (cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native table 200 $v > $GRAFT_REPO_ROOT/$O/tr_$n.log 2>&1) || exit 1
  python3 tools/rocprof_split.py $O/tr_$n/run_kernel_trace.csv > $O/tr_$n.split.csv; echo "== $v"; grep "ypass" $O/tr_$n.split.csv | head -1
done
ab() { timeout -k 10 300 python3 tools/ab.py --config native --mode table --rounds 7 --switch-calls 24 --events 0 --tune-a "$1" --tune-b "$2" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('A', d['A'], d['A_median_ms']['wall_ms'], '| B', d['B'], d['B_median_ms']['wall_ms'])"; }
ab yt_chunk=16 yt_chunk=24
ab yt_chunk=24 yt_chunk=16
