#!/bin/bash
# Pooled coefficient allocation physically contiguous (DFAMD_B_CONTIG) against the plain pooled hipMalloc.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2aw}
mkdir -p $O
DFAMD_B_CONTIG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "bitexact or golden" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for ct in 1 0 1 0; do
  DFAMD_B_CONTIG=$ct timeout -k 10 300 python tools/handle_var.py 4 >> $O/contig_$ct.jsonl 2> $O/contig_$ct.err || { echo "failed"; tail -20 $O/contig_$ct.err; exit 1; }
done
python3 -c "
import json, statistics
for ct in (0, 1):
    d=[json.loads(l) for l in open('$O/contig_%d.jsonl' % ct)]
    print('contig', ct, 'mean total', round(statistics.mean(x['total_ms'] for x in d),4), 'min', min(x['total_ms'] for x in d), 'max', max(x['total_ms'] for x in d), 'n', len(d))"
