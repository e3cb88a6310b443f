#!/bin/bash
# Table mode, where the VALU goes: SQ instruction counters per kernel of a c3 table call (two --pmc
# passes, no traces), the K3a chunks-per-wave A/B, and the cost of the per-call phase events on short
# calls (tools/event_cost.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3d}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $O/p$i -o run --output-format csv -- \
     python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 6 > $O/p$i.log 2>&1) || { echo "pmc $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O ypass zpass rng_ > $O/pmc_c3_table.json
python3 - $O/pmc_c3_table.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
tot = 0
for k, v in d.items():
    tot += v.get('SQ_INSTS_VALU', 0)
    print(k[:60].ljust(60), 'VALU %.2fM SALU %.2fM waves %d' % (v.get('SQ_INSTS_VALU', 0) / 1e6, v.get('SQ_INSTS_SALU', 0) / 1e6, v.get('SQ_WAVES', 0)))
print('total VALU per call %.1fM wave-instr' % (tot / 1e6))
PY
for g in 4 16; do
  timeout -k 10 300 python3 tools/ab.py --torch --config c3 --mode table --rounds 9 --tune-a dense_g=8 --tune-b dense_g=$g \
    > $O/ab_dense_g$g.json 2> $O/ab_g$g.err || { echo "ab failed"; tail -20 $O/ab_g$g.err; exit 1; }
  cat $O/ab_dense_g$g.json
done
for cfg in "c2 packed" "native packed" "c2 table" "native table" "c3 table"; do
  timeout -k 10 120 python3 tools/event_cost.py $cfg 9 50 >> $O/event_cost.jsonl 2> $O/ev.err || { echo "event_cost failed"; tail -5 $O/ev.err; exit 1; }
done
cat $O/event_cost.jsonl
