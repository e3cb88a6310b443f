#!/bin/bash
# Split counting with counts-only exchange (K3 recounts its waves' accept flags): parity (groups, one-rank
# RCCL, emulated-host RCCL), then one rank of a c4 split timed alone, replicated vs split, both modes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2aa}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multi.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for mode in table packed; do
  for rep in 1 0; do
    timeout -k 10 300 python tools/strip_timing.py --config c4 --mode $mode --replicate $rep --ns 4,8 --calls 30 >> $O/strip.jsonl 2>> $O/strip.err \
      || { echo "strip failed"; tail -20 $O/strip.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/strip.jsonl'):
    d=json.loads(l); print(d['mode'], 'rep', d['replicate'], 'N', d['N'], 'rank', d['rank'], 'wall', d['wall_ms'], 'rng', d['rng_ms'], 'y', d['ypass_ms'], 'z', d['zpass_ms'])"
