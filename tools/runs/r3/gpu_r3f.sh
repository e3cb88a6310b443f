#!/bin/bash
# Is the packed c3 z-pass slower with the round-3 code, or is it the box? The round-2 library
# (c5439f4, built as libdfamd_r2.so) against the current one, alternating, same box, events on
# every call for both (the r2 library has no sampled events).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3f}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
for i in 1 2; do
  for lib in r2 cur; do
    if [ $lib = r2 ]; then L=$GRAFT_REPO_ROOT/digital-filtering_amd/libdfamd_r2.so; else L=; fi
    DFAMD_LIB=$L timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --profile-every 1 --alt-modes off --other-configs '' \
      --dropin off --cpu-baseline off --parity off > $O/c3_${lib}_$i.json 2> $O/c3_${lib}_$i.err || { echo "bench $lib failed"; tail -5 $O/c3_${lib}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c3_${lib}_$i.json')); print('$lib', $i, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['phase_ms_per_call'])"
  done
done
