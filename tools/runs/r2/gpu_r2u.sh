#!/bin/bash
# Native-grid y-pass ablations (timing only): register noise, register coefficients, one-product
# cooperative sum, each with ycoop 2 (current) against ycoop 4 (pipelined), RNG overlap off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2u
mkdir -p $O
for v in "" abl_noise abl_coef abl_coopsum; do
  lib=digital-filtering_amd/libdfamd${v:+_$v}.so
  DFAMD_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a ycoop=2 --tune-b ycoop=4 \
    --config native --mode packed --rounds 7 --calls 20 > $O/ab_$v.json 2>> $O/ab.err || { echo "ab $v failed"; tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/ab_$v.json')); print('$v', d['A'], d['A_median_ms']['ypass_ms'], d['A_median_ms']['zpass_ms'], d['B'], d['B_median_ms']['ypass_ms'], d['B_median_ms']['zpass_ms'], d['B_median_ms']['wall_ms'])"
done
