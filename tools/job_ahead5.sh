set -o pipefail
# the three-epoch ahead form on the planes that do not use it by default, and c3 table's hand-off batch
cd $GRAFT_REPO_ROOT
O=gpurun_out/ahead5; mkdir -p $O
ab() { timeout -k 10 300 python3 tools/ab.py --config $1 --mode $2 --rounds ${5:-9} --switch-calls 24 --events 0 --tune-a "$3" --tune-b "$4" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['mode'], 'A', d['A'], d['A_median_ms']['wall_ms'], '| B', d['B'], d['B_median_ms']['wall_ms'])"; }
timeout -k 10 300 python3 tools/ab.py --config c3 --mode table --rounds 7 --events 0 --a DFAMD_HANDOFF_BATCH=2 --b DFAMD_HANDOFF_BATCH=4 >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | cut -c1-400
ab c2 packed ypass_ahead=0 ypass_ahead=1
ab c2 table ypass_ahead=0 ypass_ahead=1
ab c1 packed ypass_ahead=0 ypass_ahead=1
ab c1 table ypass_ahead=0 ypass_ahead=1
