set -o pipefail
# c2 packed launch shapes, one handle, 60-call windows, both orders (phase events on: the z-pass time is the line's roofline)
cd $GRAFT_REPO_ROOT
O=gpurun_out/c2; mkdir -p $O
ab() { timeout -k 10 300 python3 tools/ab.py --config c2 --mode packed --rounds 7 --switch-calls 24 --events 1 --tune-a "$1" --tune-b "$2" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); a,b=d['A_median_ms'],d['B_median_ms']; print('A', d['A'], a['wall_ms'], a['zpass_ms'], a['ypass_ms'], '| B', d['B'], b['wall_ms'], b['zpass_ms'], b['ypass_ms'])"; }
ab zsplit=0 zsplit=1
ab zsplit=1 zsplit=0
ab handoff_batch=2 handoff_batch=1
ab handoff_batch=1 handoff_batch=2
ab nt_stores=1 nt_stores=0
ab nt_stores=0 nt_stores=1
