set -o pipefail
# y-pass ahead with three epochs of noise sets: parity (ahead, multi-GPU emulated, native), steady-state A/B, trace
cd $GRAFT_REPO_ROOT
O=gpurun_out/ahead3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ahead.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_ghost.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "ahead or native_grid or runtime_tuning or ghost or emulated or hb" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
ab() { timeout -k 10 300 python3 tools/ab.py --config $1 --mode $2 --rounds 9 --switch-calls 24 --tune-a "$3" --tune-b "$4" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['mode'], 'A', d['A'], d['A_median_ms']['wall_ms'], d['A_median_ms'], '| B', d['B'], d['B_median_ms']['wall_ms'])"; }
ab native packed ypass_ahead=0 ypass_ahead=1
ab native table ypass_ahead=0 ypass_ahead=1
ab native packed ypass_ahead=1,ycoop_split=0 ypass_ahead=1,ycoop_split=96
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trp -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native packed 300 > $GRAFT_REPO_ROOT/$O/trp.log 2>&1) || exit 1
python3 tools/timeline.py $O/trp/run_kernel_trace.csv 40
timeout -k 10 400 python3 tools/strip_timing.py --config c4 --mode table --replicate 0 --ns 8 --calls 200 > $O/strip.jsonl 2> $O/strip.err || { tail $O/strip.err; exit 1; }
timeout -k 10 400 python3 tools/strip_timing.py --config c4 --mode table --replicate 0 --ns 8 --calls 200 --env DFAMD_SOLO_XCHG_US=40 >> $O/strip.jsonl 2>> $O/strip.err || { tail $O/strip.err; exit 1; }
cut -c1-200 $O/strip.jsonl
