#!/bin/bash
# One rank of an 8-way c4 split in table mode (timing only, DFAMD_SOLO_STRIP): kernel split with the RNG
# overlapped and serialized (DFAMD_RNG_OVERLAP=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2z}
mkdir -p $O
export TMPDIR=/tmp
for ov in 1 0; do
  (cd /tmp && DFAMD_RNG_OVERLAP=$ov timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ov$ov -o run -- \
     python3 $GRAFT_REPO_ROOT/tools/strip_timing.py --config c4 --mode table --ns 8 --calls 40 > $O/strip_ov$ov.jsonl 2> $O/prof_ov$ov.err) \
     || { echo "rocprof failed"; tail -5 $O/prof_ov$ov.err; exit 1; }
  cat $O/strip_ov$ov.jsonl
  python3 tools/rocprof_split.py $O/prof_ov$ov/run_kernel_trace.csv > $O/split_ov$ov.csv
  head -14 $O/split_ov$ov.csv
  rm -f $O/prof_ov$ov/run_kernel_trace.csv
done
