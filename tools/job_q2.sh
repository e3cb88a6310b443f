set -o pipefail
# order bias check of the one-handle A/B on the reference's grid, packed
cd $GRAFT_REPO_ROOT
O=gpurun_out/q2; mkdir -p $O
ab() { timeout -k 10 300 python3 tools/ab.py --config native --mode packed --rounds 7 --switch-calls 24 --events ${3:-0} --tune-a "$1" --tune-b "$2" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('A', d['A'], d['A_median_ms'], '| B', d['B'], d['B_median_ms'])"; }
ab ycoop_split4=192 ycoop_split4=193
ab ycoop_split4=0 ycoop_split4=1000
ab ycoop_split4=192 ycoop_split4=0
ab ycoop_split4=0 ycoop_split4=192 1
timeout -k 10 200 python3 tools/phase_time.py --config native --mode packed > $O/p0.json 2>&1; tail -1 $O/p0.json
timeout -k 10 200 python3 tools/phase_time.py --config native --mode packed --tune ycoop_split4=160 > $O/p1.json 2>&1; tail -1 $O/p1.json
