#!/bin/bash
# Stream priorities (sweeps high, RNG low: DFAMD_RNG_PRIO=1) on the reference's grid and c2/c3, two handles
# per A/B, run twice with A and B swapped (handle placement differs by a few %).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bb
mkdir -p $O
for cm in "native packed" "native table" "c2 packed" "c3 packed"; do
  set -- $cm
  for ord in "0 1" "1 0"; do
    set -- $cm $ord
    timeout -k 10 200 python3 tools/ab.py --config $1 --mode $2 --rounds 9 --calls 20 --a DFAMD_RNG_PRIO=$3 --b DFAMD_RNG_PRIO=$4 \
      > $O/ab_$1_$2_$3$4.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_$1_$2_$3$4.json'));print('$1 $2', d['A'], d['A_median_ms']['wall_ms'], d['B'], d['B_median_ms']['wall_ms'])"
  done
done
