#!/bin/bash
# Table-mode c3 as the bench's main line (cool GPU) vs as the alt mode after the packed run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2l
mkdir -p $O
timeout -k 10 300 python bench.py --coeff-mode table --steps 20 --warmup 5 --cpu-baseline off --other-configs '' > $O/bench_table_main.json 2> $O/err1 \
  || { echo "bench failed"; tail -20 $O/err1; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --other-configs '' > $O/bench_packed_main.json 2> $O/err2 \
  || { echo "bench failed"; tail -20 $O/err2; exit 1; }
python3 -c "
import json
a=json.load(open('$O/bench_table_main.json')); b=json.load(open('$O/bench_packed_main.json'))
print('table main', a['ms_per_step'], a['phase_ms_per_call'], 'packed alt', a['alt_modes']['packed']['ms_per_step'])
print('packed main', b['ms_per_step'], b['phase_ms_per_call'], 'table alt', b['alt_modes']['table']['ms_per_step'], b['alt_modes']['table']['phase_ms_per_call'])"
