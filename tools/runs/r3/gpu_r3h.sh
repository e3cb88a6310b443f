#!/bin/bash
# The per-call stream hand-off on small planes: wall per call with the noise wait / the release event
# ablated (timing only), c2 and the reference's grid, both modes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3h}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
for cfg in "c2 packed" "native packed" "c2 table" "native table" "c1 packed" "c3 table"; do
  timeout -k 10 200 python3 tools/handoff_ab.py $cfg 7 50 >> $O/handoff.jsonl 2>> $O/h.err || { echo "failed $cfg"; tail -20 $O/h.err; exit 1; }
  tail -1 $O/handoff.jsonl
done
