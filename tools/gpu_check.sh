#!/bin/bash
# Parity first, then the benchmark in both coefficient modes. Usage: tools/gpu_check.sh TAG [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-check}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for mode in packed table; do
  timeout -k 10 300 python bench.py --cpu-baseline off --alt-modes off --coeff-mode $mode "$@" > $O/bench_$mode.json 2> $O/bench_$mode.err || { echo "bench $mode failed"; tail -5 $O/bench_$mode.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$mode.json')); print('$mode', d['value'], d['ms_per_step'], d['phase_ms_per_call'], d['roofline']['frac'])"
done
