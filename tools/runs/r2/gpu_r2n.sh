#!/bin/bash
# Why does bench.py time table-mode c3 at ~0.43 ms/call while tools/ab.py sees ~0.36? Seed and step count.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2n
mkdir -p $O
for args in "--seed 1" "--seed 42" "--seed 1 --steps 140 --warmup 5"; do
  timeout -k 10 300 python bench.py --coeff-mode table --alt-modes off --parity off --cpu-baseline off --other-configs '' $args > $O/b.json 2> $O/err \
    || { echo "bench failed"; tail -20 $O/err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('$args', d['ms_per_step'], d['phase_ms_per_call'])"
done
