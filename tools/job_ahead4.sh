set -o pipefail
# ahead at hb 4 (12 sets) on the reference's grid: parity, steady-state A/B, trace, then the bench line
cd $GRAFT_REPO_ROOT
O=gpurun_out/ahead4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ahead.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "ahead or native_grid or runtime_tuning or hb" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
ab() { timeout -k 10 300 python3 tools/ab.py --config $1 --mode $2 --rounds 9 --switch-calls 24 --events 0 --tune-a "$3" --tune-b "$4" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['mode'], 'A', d['A'], d['A_median_ms']['wall_ms'], '| B', d['B'], d['B_median_ms']['wall_ms'])"; }
ab native packed ypass_ahead=0 ypass_ahead=1
ab native table ypass_ahead=0 ypass_ahead=1
ab native packed ypass_ahead=1,handoff_batch=4 ypass_ahead=1,handoff_batch=2
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trp -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native packed 300 > $GRAFT_REPO_ROOT/$O/trp.log 2>&1) || exit 1
python3 tools/timeline.py $O/trp/run_kernel_trace.csv 24
timeout -k 10 600 python3 bench.py --cpu-baseline off > $O/bench.json 2> $O/bench.log || exit 1
python3 tools/bench_summary.py $O/bench.json
