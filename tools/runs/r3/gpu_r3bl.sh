#!/bin/bash
# Table mode at N = 8 (its defaults: split counting, serial halo): one rank of c4 timed alone (DFAMD_SOLO_STRIP),
# phases, and the rocprofv3 kernel split of the same run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bl
mkdir -p $O
timeout -k 10 300 python3 tools/strip_timing.py --config c4 --mode table --replicate 0 --ns 8,1 --calls 40 > $O/strip_table.jsonl 2> $O/strip.err \
  || { echo "strip timing failed"; tail -20 $O/strip.err; exit 1; }
cat $O/strip_table.jsonl
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
   python3 $GRAFT_REPO_ROOT/tools/strip_timing.py --config c4 --mode table --replicate 0 --ns 8 --calls 40 > $O/prof_run.jsonl 2> $O/prof.err) \
   || { echo "rocprof failed"; tail -5 $O/prof.err; exit 1; }
python3 tools/rocprof_split.py $O/prof/run_kernel_trace.csv > $O/kernel_split.csv
head -16 $O/kernel_split.csv
rm -f $O/prof/run_kernel_trace.csv
