#!/bin/bash
# Round-3 full pass: GPU suite, smoke, the default bench line, rocprofv3 --kernel-trace --stats of the
# same command (plus the per-grid split), and c4 / c5 on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3full}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --durations=25 \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err \
  || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_default.json'))
print('c3', d['value'], d['ms_per_step'], 'parity', d['parity_ok'], 'frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'])
print('table', d['alt_modes']['table']['ms_per_step'], d['alt_modes']['table']['roofline_valu'])
print({k:(v['ms_per_step'],v['parity_ok'],v['roofline']['frac']) for k,v in (d['other_configs'] or {}).items()})
print({k:(v.get('capi_ms'), v.get('dropin_ms')) for k,v in (d.get('dropin') or {}).items()})"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
   python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --dropin off > $O/bench_under_rocprof.json 2> $O/prof.err) \
   || { echo "rocprof failed"; tail -5 $O/prof.err; exit 1; }
python3 tools/rocprof_split.py $O/prof/run_kernel_trace.csv > $O/kernel_split.csv
head -14 $O/kernel_split.csv
rm -f $O/prof/run_kernel_trace.csv
for cfg in c4 c5; do
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --cpu-baseline off --other-configs '' --alt-modes off \
    --dropin off > $O/bench_${cfg}_n1.json 2> $O/bench_${cfg}.err || { echo "bench $cfg failed"; tail -20 $O/bench_${cfg}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${cfg}_n1.json')); print('$cfg', d['value'], d['ms_per_step'], d['parity_ok'], d['roofline']['frac'])"
done
