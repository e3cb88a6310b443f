#!/bin/bash
# Table mode, c3 (and c2, the reference's grid): register budgets that leave room for the RNG beside the sweeps:
# z-pass at 7 or 8 waves per SIMD (70 / 54 VGPRs, no spills), K3a at 7 (72 VGPRs, 44 B spilled); libraries
# alternated, separate processes. The packed z-pass shares the template: c3 packed timed too.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ab
mkdir -p $O
L=$GRAFT_REPO_ROOT/digital-filtering_amd
for i in 1 2; do
  for v in "" _zw7 _zw8 _k3w7 _zw8k3w7; do
    DFAMD_LIB=$L/libdfamd$v.so timeout -k 10 120 python3 tools/ab.py --config c3 --mode table --rounds 7 --calls 20 \
      > $O/lib${v}_$i.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/lib${v}_$i.json'));print('c3 table lib$v', d['A_median_ms'], d['B_median_ms']['wall_ms'])"
  done
done
for v in "" _zw8; do
  for cm in "c2 table" "native table" "c3 packed"; do
    set -- $cm
    DFAMD_LIB=$L/libdfamd$v.so timeout -k 10 120 python3 tools/ab.py --config $1 --mode $2 --rounds 7 --calls 20 \
      > $O/lib${v}_$1_$2.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/lib${v}_$1_$2.json'));print('$1 $2 lib$v', d['A_median_ms']['wall_ms'], d['B_median_ms']['wall_ms'])"
  done
done
