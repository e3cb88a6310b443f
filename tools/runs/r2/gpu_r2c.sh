#!/bin/bash
# Compacted K3: standalone time under timing-only ablations (DFAMD_RNG_DEBUG: 1 no log/sqrt/div,
# 2 no stores, 4 no redraw; wrong results by design, parity off) and its PMC counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r2c
mkdir -p $O
export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --coeff-mode table --cpu-baseline off --alt-modes off --other-configs '' --parity off --steps 20 --warmup 3"
for f in 0 1 2 4 7; do
  (cd /tmp && DFAMD_RNG_OVERLAP=0 DFAMD_RNG_DEBUG=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv \
     -d $O/abl$f -o run -- python3 $GRAFT_REPO_ROOT/bench.py --coeff-mode table --cpu-baseline off --alt-modes off \
     --other-configs '' --parity off --steps 20 --warmup 3 > $O/abl$f.log 2>&1) || { echo "ablation $f failed"; tail -5 $O/abl$f.log; exit 1; }
  python3 - "$O/abl$f/run_kernel_stats.csv" $f <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if 'rng_generate' in x['Name'] or 'rng_count' in x['Name']:
        print('flags', sys.argv[2], '%-40s avg_us=%9.1f' % (x['Name'][:40], float(x['AverageNs']) / 1e3))
PY
done
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  (cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $O/pmc$i -o run --output-format csv -- \
     python3 $GRAFT_REPO_ROOT/bench.py --coeff-mode table --cpu-baseline off --alt-modes off --other-configs '' --parity off --steps 5 --warmup 1 \
     > $O/pmc$i.log 2>&1) || { echo "pmc $i failed"; tail -5 $O/pmc$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O rng_generate rng_count > $O/pmc_summary.json && cat $O/pmc_summary.json
