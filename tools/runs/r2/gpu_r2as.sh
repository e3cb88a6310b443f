#!/bin/bash
# Spread of the packed c3 sweeps between handles alive at once (5 handles x 21 GB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2as}
mkdir -p $O
timeout -k 10 400 python tools/handle_var.py 5 > $O/handles.jsonl 2> $O/handles.err || { echo "failed"; tail -20 $O/handles.err; exit 1; }
cat $O/handles.jsonl
