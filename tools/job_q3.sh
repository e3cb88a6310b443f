set -o pipefail
# one-handle A/B with 60-call windows (the ahead pipeline holds ~2 epochs of work: 10-call windows mis-time it)
cd $GRAFT_REPO_ROOT
O=gpurun_out/q3; mkdir -p $O
ab() { timeout -k 10 300 python3 tools/ab.py --config $1 --mode $2 --rounds 7 --calls 60 --switch-calls 24 --events 0 --tune-a "$3" --tune-b "$4" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['mode'], 'A', d['A'], d['A_median_ms']['wall_ms'], '| B', d['B'], d['B_median_ms']['wall_ms'])"; }
ab native packed ycoop_split4=192 ycoop_split4=193
ab native packed ypass_ahead=0 ypass_ahead=1
ab native packed ypass_ahead=1 ypass_ahead=0
ab native table ypass_ahead=0 ypass_ahead=1
ab native table ypass_ahead=1 ypass_ahead=0
ab native packed ycoop_split4=0 ycoop_split4=192
ab native packed ycoop_split4=192 ycoop_split4=0
ab native packed ycoop_split=96 ycoop_split=0
ab native packed ycoop_split=0 ycoop_split=96
