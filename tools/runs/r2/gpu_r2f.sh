#!/bin/bash
# Native-grid vs c2 packed y-pass counters (RNG overlap off): HBM bytes, L2 hits/misses, waves.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2f; mkdir -p $O
for plane in native c2; do
  i=0
  for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM" "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum" "GRBM_GUI_ACTIVE TCC_EA0_RDREQ_32B_sum"; do
    i=$((i+1))
    DFAMD_RNG_OVERLAP=0 timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $O/${plane}_p$i -o run --output-format csv -- \
      python3 $R/tools/plane_loop.py $plane packed 6 > $O/${plane}_p$i.log 2>&1 || { echo "pass $plane $i failed"; tail -3 $O/${plane}_p$i.log; exit 1; }
  done
  python3 $R/tools/pmc_summary.py $O ypass > $O/summary_$plane.json
  rm -rf $O/${plane}_p*
  python3 -c "
import json; d=json.load(open('$O/summary_$plane.json'))
for k,v in d.items(): print('$plane', k, {c: (round(x/1e6,3) if isinstance(x,float) else x) for c,x in v.items()})"
done
