set -o pipefail
# row-pair y-pass: wide-stencil tiles as two 64-column halves (ycoop_split N threshold), parity then A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out/split; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "native_grid or runtime_tuning" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
ab() { timeout -k 10 300 python3 tools/ab.py --config native --mode packed --rounds 9 --switch-calls 3 --tune-a "$1" --tune-b "$2" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('A', d['A'], d['A_median_ms'], '| B', d['B'], d['B_median_ms'])"; }
ab ycoop_split=0 ycoop_split=160
ab ycoop_split=0 ycoop_split=128
ab ycoop_split=0 ycoop_split=96
ab ycoop_split=0 ycoop_split=64
ab ycoop_split=0 ycoop_split=1
ab ycoop_split=0,ypass_ahead=0 ycoop_split=96,ypass_ahead=0
(cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr0 -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native packed 100 ycoop_split=0 > $GRAFT_REPO_ROOT/$O/tr0.log 2>&1) || exit 1
(cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr96 -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native packed 100 ycoop_split=96 > $GRAFT_REPO_ROOT/$O/tr96.log 2>&1) || exit 1
for t in tr0 tr96; do python3 tools/rocprof_split.py $O/$t/run_kernel_trace.csv > $O/$t.split.csv; echo "== $t"; grep ypass $O/$t.split.csv | head -2; done
