#!/bin/bash
# Table y-pass occupancy: waves-per-EU hints 5 and 6 (libdfamd_wpe5/6.so, timing builds) against the default
# (4 waves per SIMD at 123 VGPRs); c3 table, RNG overlap off and on; libraries alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3z
mkdir -p $O
L=$GRAFT_REPO_ROOT/digital-filtering_amd
for i in 1 2; do
  for v in "" _wpe5 _wpe6; do
    for ov in 0 1; do
      DFAMD_LIB=$L/libdfamd$v.so DFAMD_RNG_OVERLAP=$ov timeout -k 10 120 python3 tools/ab.py --config c3 --mode table --rounds 7 --calls 20 \
        > $O/ab${v}_ov${ov}_$i.json || { echo "ab failed"; exit 1; }
      python3 -c "import json;d=json.load(open('$O/ab${v}_ov${ov}_$i.json'));print('lib$v overlap $ov', d['A_median_ms'])"
    done
  done
done
