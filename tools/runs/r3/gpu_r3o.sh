#!/bin/bash
# Row-pair y-pass sum: LDS reads batched 8 at a time (default) vs one LDS round trip per add
# (libdfamd_serialsum.so, -DDF_COOP2_SERIAL_SUM), on the reference's grid, packed; libraries alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3o
mkdir -p $O
L=$GRAFT_REPO_ROOT/digital-filtering_amd
for i in 1 2 3; do
  for lib in libdfamd.so libdfamd_serialsum.so; do
    DFAMD_LIB=$L/$lib timeout -k 10 120 python3 tools/ab.py --config native --mode packed --rounds 9 --calls 20 \
      > $O/ab_${lib%.so}_$i.json || { echo "ab $lib failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_${lib%.so}_$i.json'));print('$lib', d['A_median_ms'], d['B_median_ms']['ypass_ms'])"
  done
done
