#!/bin/bash
# Table-mode launch shapes re-checked after the loads-first z staging and glibc_log (c3, RNG overlapped).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2aq}
mkdir -p $O
for t in "zunroll=4 zunroll=2" "heavy_first=1 heavy_first=0" "rows_per_wave=4 rows_per_wave=2" "gen_split=1 gen_split=2" "nt_stores=1 nt_stores=0" "rng_nt_stores=1 rng_nt_stores=0"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --tune-a $1 --tune-b $2 --config c3 --mode table --rounds 9 --calls 30 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); a=d['A_median_ms']; b=d['B_median_ms']; print(d['config'], d['mode'], d['A'], a.get('ypass_ms'), a.get('zpass_ms'), a['wall_ms'], '|', d['B'], b.get('ypass_ms'), b.get('zpass_ms'), b['wall_ms'])"
