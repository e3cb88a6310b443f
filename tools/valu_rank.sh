#!/bin/bash
# VALU/SALU wave-instructions per kernel of one c4/8 table rank (solo strip, tools/solo_rank.py), one PMC pass
# (SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU, kernel trace only) -> gpurun_out/valu_rank<R>/pmc.json.
#   bash tools/valu_rank.sh RANK [--tune k=v:k=v]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
RANK=${1:-0}; shift
O=$R/gpurun_out/valu_rank$RANK; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace -d $O/p1 -o run --output-format csv -- \
   python3 $R/tools/solo_rank.py --N 8 --rank $RANK --calls 8 "$@" > $O/p1.log 2>&1 || { echo "pmc failed"; tail -5 $O/p1.log; exit 1; }
python3 $R/tools/pmc_summary.py $O ypass zpass rng_ replicate > $O/pmc.json
python3 - $O/pmc.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
tot = 0
for k, v in d.items():
    tot += v.get("SQ_INSTS_VALU", 0)
    print(f"{k[:60]:60s} VALU {v.get('SQ_INSTS_VALU', 0)/1e6:7.2f}M  SALU {v.get('SQ_INSTS_SALU', 0)/1e6:7.2f}M  waves {v.get('SQ_WAVES', 0):.0f}")
print(f"total VALU per call {tot/1e6:.1f}M")
PY
