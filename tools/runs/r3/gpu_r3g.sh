#!/bin/bash
# Small planes: is the per-call K5 -> K4 hand-off the cross-stream RNG event? c2 and the reference's
# grid, packed and table, RNG on its own stream (default) against serial on the main stream; then the
# default bench line for the new table-mode call-issue roofline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3g}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
for cfg in "c2 packed" "native packed" "c2 table" "native table"; do
  set -- $cfg
  timeout -k 10 300 python3 tools/ab.py --torch --config $1 --mode $2 --rounds 9 --calls 40 --a "" --b DFAMD_RNG_OVERLAP=0 \
    >> $O/ab_overlap_small.jsonl 2>> $O/ab.err || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
  tail -1 $O/ab_overlap_small.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['mode'], 'overlap', d['A_median_ms']['wall_ms'], 'serial', d['B_median_ms']['wall_ms'])"
done
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --dropin off > $O/bench_default.json 2> $O/bench_default.err \
  || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_default.json'))
print('c3', d['value'], d['ms_per_step'], 'frac', d['roofline']['frac'])
print('table', d['alt_modes']['table']['ms_per_step'], d['alt_modes']['table']['roofline_valu'].get('call_issue'))
print({k:(v['ms_per_step'],v['parity_ok'],v['roofline']['frac']) for k,v in (d['other_configs'] or {}).items()})"
