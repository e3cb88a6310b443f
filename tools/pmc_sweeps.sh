#!/bin/bash
# rocprofv3 counters of the sweeps (separate --pmc passes, kernel trace only) on a 1-GPU
# plane: tools/solo_rank.py 1 0 MODE 4. Usage: tools/pmc_sweeps.sh [table|packed]
# Summarize with tools/pmc_summary.py gpurun_out/pmcsw_MODE.
MODE=${1:-table}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcsw_$MODE; mkdir -p $O
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES" "SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  DFAMD_RNG_OVERLAP=0 timeout -k 10 240 rocprofv3 --pmc $set --kernel-trace -d $O/p$i -o run --output-format csv -- python3 $R/tools/solo_rank.py 1 0 $MODE 4 > $O/p$i.log 2>&1
  rc=$?
  echo "pass $i ($set): rc=$rc"
  case $rc in 124|134|137|139) echo "stopping after rc=$rc"; exit $rc;; esac
done
