#!/bin/bash
# Cost of the split z-pass (interior strips on the stream, edge strips on the high-priority comm_stream)
# without any exchange: one rank of a c4 split over 8 (and 4) timed alone (DFAMD_SOLO_STRIP), halo_overlap
# 1 vs 0, packed and table. The xGMI gain is the exchange time minus this difference.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3az
mkdir -p $O
for mode in packed table; do
  for ov in 0 1 0 1; do
    timeout -k 10 300 python3 tools/strip_timing.py --config c4 --mode $mode --ns 8,4 --calls 40 --tune halo_overlap=$ov \
      >> $O/strip_c4_$mode.jsonl 2>> $O/strip.err || { echo "strip timing $mode ov$ov failed"; tail -20 $O/strip.err; exit 1; }
  done
done
cat $O/strip_c4_*.jsonl
