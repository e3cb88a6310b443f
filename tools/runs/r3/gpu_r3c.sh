#!/bin/bash
# Full pass with dense generation as the table default: GPU suite (incl. emulated worlds 2-8 and the
# c5 eight-strip groups), smoke, default bench, the c5 10k-step long run on one GPU, and a bare
# `bench.py --gpus 4` with emulated hosts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3c}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
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
print({k:(v['ms_per_step'],v['parity_ok'],v['roofline']['frac']) for k,v in (d['other_configs'] or {}).items()})"
timeout -k 10 400 python bench.py --config c5 --steps 10 --warmup 3 --long-run 10000 --other-configs '' --alt-modes off \
  --dropin off --cpu-baseline off > $O/bench_c5_long.json 2> $O/bench_c5_long.err \
  || { echo "c5 long failed"; tail -20 $O/bench_c5_long.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_c5_long.json')); print('c5', d['ms_per_step'], d['parity_ok'], json.dumps(d['long_run']))"
DFAMD_EMULATE_HOSTS=1 timeout -k 10 600 python3 bench.py --gpus 4 --steps 10 --warmup 3 --other-configs '' \
  --long-run 0 > $O/bench_emu_n4.json 2> $O/bench_emu_n4.err \
  || { echo "emulated bench failed"; tail -40 $O/bench_emu_n4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_emu_n4.json').read().strip())
m=d['multi_gpu']; print('emu n4', d['n_gpus'], 'rccl', m['rccl_ranks'], 'parity', d['parity_ok'], d['ms_per_step'], 'same', d.get('ms_per_step_1gpu_same_plane'), d.get('speedup'))"
