#!/bin/bash
# Hand-off batching re-measured on the reference's grid after this round's y-pass changes (tools/hb_ab.py: one
# handle per hb 1/2/4 and burst forms, interleaved rounds, no phase events), packed and table; twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3at
mkdir -p $O
for mode in packed table; do
  for i in 1 2; do
    timeout -k 10 300 python3 tools/hb_ab.py native $mode 9 48 >> $O/hb_native_$mode.jsonl || { echo "hb_ab failed"; exit 1; }
    tail -1 $O/hb_native_$mode.jsonl
  done
done
