#!/bin/bash
# rocprofv3 counters of the RNG kernels (separate --pmc passes, no traces), one z-strip rank
# of an N-way split on one GPU (tools/solo_rank.py). Usage: tools/pmc_rng.sh N [packed|table]
set -e
N=${1:-1}; MODE=${2:-table}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcrng_n$N; mkdir -p $O
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES" "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"; do
  i=$((i+1))
  DFAMD_RNG_OVERLAP=0 timeout -k 10 240 rocprofv3 --pmc $set --kernel-trace -d $O/p$i -o run --output-format csv -- python3 $R/tools/solo_rank.py $N 0 $MODE 4 > $O/p$i.log 2>&1
done
echo done
