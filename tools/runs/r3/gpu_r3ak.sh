#!/bin/bash
# Sweeps' wave issue priority (s_setprio, sweep_prio 0 vs 1 / 3) with the next call's RNG resident beside them:
# same handle, c2/native/c3 packed and c3 table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ak
mkdir -p $O
for cm in "c2 packed" "native packed" "c3 packed" "c3 table" "native table"; do
  set -- $cm
  for p in 1 3; do
    timeout -k 10 200 python3 tools/ab.py --config $1 --mode $2 --rounds 9 --calls 20 --tune-a sweep_prio=0 --tune-b sweep_prio=$p \
      > $O/ab_$1_$2_p$p.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_$1_$2_p$p.json'));print('$1 $2 prio0', d['A_median_ms'], 'prio$p', d['B_median_ms'])"
  done
done
