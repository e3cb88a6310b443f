set -o pipefail
# y-pass ahead: parity, then same-handle A/B on every plane of the N=1 line
cd $GRAFT_REPO_ROOT
O=gpurun_out/ahead; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ahead.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "ahead or runtime_tuning or stage_api" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
ab() { timeout -k 10 300 python3 tools/ab.py --config $1 --mode $2 --rounds ${3:-9} --switch-calls 12 --tune-a ypass_ahead=0 --tune-b ypass_ahead=1 >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['mode'], 'A', d['A_median_ms'], '| B', d['B_median_ms'])"; }
ab native table
ab native packed
ab c1 packed
ab c2 packed
ab c3 table
ab c3 packed 5
