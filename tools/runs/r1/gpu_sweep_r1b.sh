#!/bin/bash
# Round-1 tuning sweep on one MI355X: parity first, then HBM probe and bench variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1b
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 tools/hbm_probe 8 > $O/hbm_probe.json || exit 1
cat $O/hbm_probe.json
for v in "packed 8 0" "packed 8 1" "packed 4 0" "packed 4 1" "table 8 0" "table 4 0"; do
  set -- $v
  DFAMD_NT_LOADS=$3 timeout -k 10 300 python bench.py --cpu-baseline off --coeff-mode $1 --rows-per-wave $2 --steps 40 > $O/bench_$1_r$2_nt$3.json 2>$O/bench_$1_r$2_nt$3.err || { echo "bench $v failed"; tail -5 $O/bench_$1_r$2_nt$3.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$1_r$2_nt$3.json')); print('$v', d['value'], d['ms_per_step'], d['phase_ms_per_call'], d['roofline']['frac'])"
done
