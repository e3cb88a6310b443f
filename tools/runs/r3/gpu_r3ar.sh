#!/bin/bash
# Packed mode with the dense generation (Kc + K3a fast chunks: fewer RNG instructions beside the HBM-bound sweeps,
# +16 B per stored pair of state traffic) vs the compacted K3 (packed default); same handle, c3 x3, c5, c2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ar
mkdir -p $O
for cfg in c3 c3 c3 c5 c2; do
  timeout -k 10 300 python3 tools/ab.py --config $cfg --mode packed --rounds 9 --calls 10 \
    --tune-a gen_dense=0 --tune-b gen_dense=1 > $O/ab_${cfg}.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_${cfg}.json'));print('$cfg compact', d['A_median_ms'], 'dense', d['B_median_ms'])"
done
