set -o pipefail
# packed z-pass: 8 vs 16 taps per step (zunroll), with and without a wave per component; parity of the switch
cd $GRAFT_REPO_ROOT
O=gpurun_out/zu; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "runtime_tuning" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
ab() { timeout -k 10 300 python3 tools/ab.py --config $1 --mode packed --rounds ${4:-9} --tune-a "$2" --tune-b "$3" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], 'A', d['A'], d['A_median_ms'], '| B', d['B'], d['B_median_ms'])"; }
ab c2 zunroll=4,zsplit=0 zunroll=8,zsplit=0
ab c2 zunroll=4,zsplit=1 zunroll=8,zsplit=1
ab c2 zunroll=4,zsplit=0 zunroll=8,zsplit=1
ab native zunroll=4 zunroll=8
ab c3 zunroll=4 zunroll=8 5
