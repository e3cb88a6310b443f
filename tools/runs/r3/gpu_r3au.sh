#!/bin/bash
# Hand-off batch on c2 (its default hb 2) and c1 (4): hb 1/2/4 and burst forms, twice, packed and table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3au
mkdir -p $O
for cfg in c2 c1; do
  for mode in packed table; do
    timeout -k 10 300 python3 tools/hb_ab.py $cfg $mode 9 48 >> $O/hb_$cfg.jsonl || { echo "hb_ab failed"; exit 1; }
    tail -1 $O/hb_$cfg.jsonl
  done
done
