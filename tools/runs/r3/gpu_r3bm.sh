#!/bin/bash
# Table mode, one rank of c4 over 8 (and 4): RNG stream at high priority (DFAMD_RNG_PRIO=2, a timing knob since
# reverted: profiles/r3/rejected/rng_prio_split) vs default, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bm
mkdir -p $O
for p in 0 2 0 2; do
  DFAMD_RNG_PRIO=$p timeout -k 10 300 python3 tools/strip_timing.py --config c4 --mode table --replicate 0 --ns 8,4 --calls 40 \
    --tune "" | sed "s/^{/{\"prio\": $p, /" >> $O/strip_prio.jsonl || { echo "strip timing failed"; exit 1; }
done
cat $O/strip_prio.jsonl
