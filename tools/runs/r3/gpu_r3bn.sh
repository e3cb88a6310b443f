#!/bin/bash
# BASELINE configs[4] on one GPU with the final library: c5 (4096^2), 10 000 filter(dt) calls with the device
# get_rms accumulation, in packed and table mode (steady state, total, the row-variance invariant).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bn
mkdir -p $O
for mode in table packed; do
  timeout -k 10 500 python3 bench.py --config c5 --coeff-mode $mode --steps 10 --warmup 3 --long-run 10000 --cpu-baseline off \
    --other-configs '' --alt-modes off --dropin off > $O/c5_long_$mode.json 2> $O/c5_long_$mode.err \
    || { echo "long run $mode failed"; tail -20 $O/c5_long_$mode.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c5_long_$mode.json').read().strip()); l=d['long_run']
print('$mode', d['ms_per_step'], d['parity_ok'], {k: l[k] for k in ('steps','total_s','steady_ms_per_call','max_rel_dev_rowvar_vs_R','fields_finite')})"
done
