set -o pipefail
# small packed planes: launch-shape A/B on one handle (phase medians), c2 and the reference's grid
cd $GRAFT_REPO_ROOT
O=gpurun_out/small; mkdir -p $O
ab() { timeout -k 10 200 python3 tools/ab.py --config $1 --mode packed --tune-a "$2" --tune-b "$3" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], 'A', d['A'], d['A_median_ms'], '| B', d['B'], d['B_median_ms'])"; }
ab c2 zsplit=0 zsplit=1
ab c2 nt_stores=1 nt_stores=0
ab c2 rows_per_wave=2 rows_per_wave=4
ab c2 yunroll=2 yunroll=4
ab c2 rows_per_wave=2 rows_per_wave=1,yunroll=8
ab native ycoop_order=4 ycoop_order=0
ab native ycoop_order=4 ycoop_order=8
ab native nt_stores=1 nt_stores=0
ab native ycoop=7 ycoop=0,rows_per_wave=2
ab native zsplit=0 zsplit=1
