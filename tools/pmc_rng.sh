set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcrng
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES" "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64" "SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_LDS" "GRBM_GUI_ACTIVE SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  DFAMD_RNG_OVERLAP=0 timeout -k 10 240 rocprofv3 --pmc $set --kernel-trace -d $R/gpurun_out/pmcrng/p$i -o run --output-format csv -- python3 $R/tools/phase_time.py --rounds 1 --calls 3 > $R/gpurun_out/pmcrng/p$i.log 2>&1
done
echo done
