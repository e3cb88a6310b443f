#!/bin/bash
# Packed c3 write windows and store/load policies re-checked with the round-2 code.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2ar}
mkdir -p $O
for t in "zwin_T=4096,zwin_W=256 zwin_T=2048,zwin_W=128" "zwin_T=4096,zwin_W=256 zwin_T=4096,zwin_W=512" \
         "ywin_T=4096,ywin_W=256 ywin_T=2048,ywin_W=256" "zwin_T=4096 zwin_T=0" "rows_per_wave=2 rows_per_wave=4" \
         "zunroll=4 zunroll=2"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --tune-a $1 --tune-b $2 --config c3 --mode packed --rounds 7 --calls 12 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); a=d['A_median_ms']; b=d['B_median_ms']; print(d['config'], d['mode'], d['A'], a.get('ypass_ms'), a.get('zpass_ms'), a['wall_ms'], '|', d['B'], b.get('ypass_ms'), b.get('zpass_ms'), b['wall_ms'])"
